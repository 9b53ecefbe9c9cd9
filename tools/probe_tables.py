"""u32 softmax tables for the probes (tools/enc_phase_probe.py, tools/dec_phase_probe.py)
from ONE torch generator.  synth.softmax_tables seeds a generator per step, and at 4096
steps that crashed torch.randn in the host under rocprofv3 --pmc (SIGSEGV); the probes
only need tables of the right shape and statistics, not synth's exact values."""


def one_generator_tables(T, B, V, device, seed=1234, sigma=3.0, scale_bits=31):
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    p = torch.softmax(sigma * torch.randn((T, B, V), generator=g, device=device, dtype=torch.float32).double(), -1)
    q = torch.clamp(torch.floor(p * float(1 << scale_bits)), min=1).to(torch.int64)
    del p
    cdf = torch.cumsum(q, -1)
    u = torch.rand((T, B), generator=g, device=device, dtype=torch.float64)
    tgt = torch.minimum((u * cdf[..., -1].double()).floor().long(), cdf[..., -1] - 1)
    sym = torch.searchsorted(cdf, tgt.unsqueeze(-1), right=True).squeeze(-1).to(torch.int32)
    return q.to(torch.int32), sym
