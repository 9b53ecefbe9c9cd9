"""Which straight 64-step form of the split-path encoder (lac_amd/csrc/lac_encode.hip
k_encode, LAC_ENC_STRAIGHT) each block of a fixture takes when coded untraced -- a
restatement of the kernel's block test for the tests, so they can show that reference-run
fixtures reach every form.

A block of <= 64 steps goes straight when every row has 0 < T < 2^62 (u64 kernel; the
u32 kernel also T <= 2^(prec-1) and T < 2^32), a positive width at its symbol and an
in-range symbol (ceil mapping), prec <= 61, and the state's width lies in
(2^(prec-1), 2^prec] -- true at every block start, since every renormalised state's
width does.  The u64 kernel picks its instance by whether every total is below 2^32
("t32" / "wide") and whether some row's total exceeds 2^(prec-1) ("ft": such a row can
take fudged_dist, arith_code.py:84, and a fudged step leaves the straight loop for the
general one: "exit").
"""
from oracle import restate


def forms_reached(rows, syms, prec, storage_bits):
    """Set of form names the blocks of this stream take: 'u32' (u32 kernel), 't32',
    't32+ft', 'wide', 'wide+ft', plus 't32+ft+exit' / 'wide+ft+exit' for blocks whose
    straight loop met a fudged step."""
    half = 1 << (prec - 1)
    denom = 1 << prec
    n = len(syms)
    R = restate._Rows(rows)
    l, h = 0, denom - 1
    out = set()
    for g0 in range(0, n, 64):
        blk = range(g0, min(n, g0 + 64))
        info = []
        for i in blk:
            cdf, minp = R.get(i)
            T, s = cdf[-1], syms[i]
            lo = cdf[s - 1] if s > 0 else 0
            info.append((T, minp, 0 <= s < len(cdf) and cdf[s] > lo))
        ok = prec <= 61 and all(0 < T < (1 << 62) and pos for T, _, pos in info)
        form = None
        if storage_bits == 32:
            if ok and all(T <= half and T < (1 << 32) for T, _, _ in info):
                form = "u32"
        elif ok:
            form = ("t32" if all(T < (1 << 32) for T, _, _ in info) else "wide") + \
                   ("+ft" if any(T > half for T, _, _ in info) else "")
        if form:
            out.add(form)
        exited = form is None
        for k, i in enumerate(blk):
            cdf, minp = R.get(i)
            w = h - l + 1
            fudged = cdf[-1] > w * minp
            if fudged and not exited and form and form.endswith("+ft"):
                out.add(form + "+exit")
                exited = True                     # the general loop takes the rest of the block
            lo, hi = restate.symbol_to_range(cdf, minp, syms[i], w)
            h = l + hi - 1
            l += lo
            while (h - l) < half:
                b = l // half
                l = l * 2 - b * denom
                h = h * 2 + 1 - b * denom
    return out
