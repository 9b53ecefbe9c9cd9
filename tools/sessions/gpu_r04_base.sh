#!/bin/bash
# Round 4 baselines for the decode work: bf16 logits decode
# stats + k_q1_decode at c3 / c4 / Qwen2 / Llama-4 vocabularies, the c2 pmf decode
# (one stream x 4096 steps) with a rocprofv3 kernel trace.
#   gpurun -- bash tools/sessions/gpu_r04_base.sh [outdir]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
o=gpurun_out/${1:-r04base}; mkdir -p $o
B="python3 bench.py --cpu-baseline off --steps 10 --warmup 5 --decode-reps 5"
for V in 32000 128256 151936 202048; do
  timeout -k 10 300 $B --input logits-bf16 --vocab $V --tokens 16 > $o/bf16_$V.json 2> $o/bf16_$V.err || exit 3
done
timeout -k 10 300 python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 3 --warmup 1 --decode-reps 3 > $o/c2.json 2> $o/c2.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/c2prof -o c2 -- python3 bench.py --cpu-baseline off --streams 1 --tokens 4096 --steps 2 --warmup 1 --decode-reps 1 > $o/c2prof.log 2>&1 || exit 3
python3 - "$o" <<'PY'
import json, sys, glob, os
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e); continue
    dec = d["parity"]["decode"]
    print(os.path.basename(f), f"enc {d['value']/1e6:.2f} M/s frac {d['roofline']['frac']:.3f}",
          f"dec {dec['symbols_per_s']/1e6:.2f} M/s", {k: round(v * 1e3, 1) for k, v in dec["kernel_ms_per_step_each"].items()},
          "rt", d["parity"]["round_trip_all_streams"])
PY
