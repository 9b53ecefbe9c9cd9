#!/usr/bin/env python3
"""Per-job device time over a long run of back-to-back jobs (tuning aid): shows how
the encode kernel's time drifts under sustained load (clock / power management),
with rocm-smi power and clock samples taken between batches of jobs.

    python tools/drift_probe.py [--input pmf|logits-bf16] [--vocab 32000] [--jobs 200]
"""
import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def smi():
    try:
        r = subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--showtemp", "--json"],
                           capture_output=True, text=True, timeout=20)
        d = json.loads(r.stdout)
        card = d[sorted(d)[0]]
        keep = {}
        for k, v in card.items():
            kl = k.lower()
            if "power" in kl or "sclk" in kl or "mclk" in kl or "temperature" in kl:
                keep[k] = v
        return keep
    except Exception as e:                                 # diagnostics only
        return {"error": str(e)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--streams", type=int, default=4096)
    ap.add_argument("--tokens", type=int, default=16)
    ap.add_argument("--input", default="pmf")
    ap.add_argument("--jobs", type=int, default=200)
    ap.add_argument("--batch", type=int, default=20, help="jobs between smi samples")
    a = ap.parse_args()
    import torch
    from lac_amd import synth
    from lac_amd.batch import BatchCoder
    dev = torch.device("cuda", 0)
    V, B, T = a.vocab, a.streams, a.tokens
    coder = BatchCoder(V, B, prec=48, capacity_bits=T * 50 + 256, device=dev)
    if a.input == "pmf":
        x, sym = synth.softmax_tables(T, B, V, seed=1234, device=dev, scale_bits=31)
        job = lambda: coder.encode_job(x, sym)
    else:
        dt = torch.bfloat16 if a.input == "logits-bf16" else torch.float32
        x, sym = synth.logits_batch(T, B, V, device=dev, dtype=dt, quantise=coder.quantize_logits)
        job = lambda: coder.encode_logits_job(x, sym)
    torch.cuda.synchronize()
    print(json.dumps({"smi_idle": smi()}), flush=True)
    s = torch.cuda.current_stream(dev)
    done = 0
    while done < a.jobs:
        n = min(a.batch, a.jobs - done)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        ev[0].record(s)
        for i in range(n):
            job()
            ev[i + 1].record(s)
        torch.cuda.synchronize()
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]
        print(json.dumps({"jobs": [done, done + n], "ms": [round(m, 4) for m in ms], "smi": smi()}), flush=True)
        done += n


if __name__ == "__main__":
    main()
