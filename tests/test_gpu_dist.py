"""The RCCL branch of the bitstream exchange (lac_amd/dist.py) on
the GPU, with a real BatchCoder: a one-rank nccl group (RCCL refuses two ranks
on one GPU -- "Duplicate GPU detected", tools/nccl_probe.py -- and the pool's
boxes have one MI355X).  Under nccl the root's own share is a P2P send to
itself in the same batch as every other rank's, so this runs every line of the
nccl path: the asynchronous all-gather of the sizes, the side stream and its
events, the pinned copy, batch_isend_irecv, and slot reuse at depth 2 and 3.
The multi-rank ordering is covered by the gloo world-2/4/8 tests (test_dist.py),
which take the same deferred path."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_world1():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    yield dev
    dist.destroy_process_group()


def _job(coder, j, T, B, V):
    from lac_amd import synth
    pmf, sym = synth.make_batch(300 + j, T, B, V, "zeros" if j % 2 else "loguniform")
    dev = coder.device
    coder.encode_job(torch.from_numpy(pmf.view(np.int32)).to(dev), torch.from_numpy(sym).to(dev))
    return coder.bits_tensor().clone(), coder.nbits_tensor().clone(), pmf, sym


@pytest.mark.parametrize("depth,jobs", [(2, 5), (3, 7)])
def test_rccl_gatherer_world1_real_coder(nccl_world1, depth, jobs):
    from lac_amd.batch import BatchCoder
    from lac_amd.dist import BitstreamGatherer
    V, B, T = 1000, 96, 10
    coder = BatchCoder(V, B, prec=48, capacity_bits=T * 50 + 256, device=nccl_world1)
    g = BitstreamGatherer(coder, depth=depth)
    assert not g.gloo and g.self_p2p
    made, seen = [], []
    for j in range(jobs):
        bits, nbits, _, _ = _job(coder, j, T, B, V)
        made.append((bits, nbits))
        g.submit()                                   # the next job's encode is enqueued behind it
        if g.last is not None:
            b, n = g.last_unpacked()
            seen.append((g.last_job, b.clone(), n.clone()))
    g.drain()
    b, n = g.last_unpacked()
    seen.append((g.last_job, b, n))
    assert [s[0] for s in seen] == list(range(1, jobs - depth + 1)) + [jobs]
    for j, b, n in seen:
        want_b, want_n = made[j - 1]
        assert torch.equal(n, want_n)
        nb = ((want_n + 7) // 8).tolist()
        for r in range(B):
            assert torch.equal(b[r, :nb[r]], want_b[r, :nb[r]]) and not b[r, nb[r]:].any()
    assert g.jobs == jobs and g.payload_bytes > 0
    coder.close()


def test_rccl_gather_and_scatter_world1_decode(nccl_world1):
    """gather_bitstreams / scatter_bitstreams over RCCL hand a coder's streams back
    unchanged, and the scattered shard decodes to the job's symbols."""
    from lac_amd.batch import BatchCoder
    from lac_amd.dist import gather_bitstreams, scatter_bitstreams
    V, B, T = 1000, 64, 8
    coder = BatchCoder(V, B, prec=48, capacity_bits=T * 50 + 256, device=nccl_world1)
    bits, nbits, pmf, sym = _job(coder, 11, T, B, V)
    ab, an = gather_bitstreams(bits, nbits)
    assert torch.equal(an, nbits) and ab.is_cuda
    sb, sn = scatter_bitstreams(ab, an, total_streams=B, device=nccl_world1)
    assert torch.equal(sn, nbits)
    stride = (sb.shape[1] + 7) // 8 * 8
    buf = torch.zeros((B, stride), dtype=torch.uint8, device=nccl_world1)
    buf[:, :sb.shape[1]] = sb
    coder.decode_open(buf, sn)
    out = coder.decode(torch.from_numpy(pmf.view(np.int32)).to(nccl_world1))
    assert torch.equal(out.cpu(), torch.from_numpy(sym))
    coder.close()


@pytest.mark.parametrize("hdr", [2, 4])
def test_pack_bits_kernel_equals_torch_packing(nccl_world1, hdr):
    """lac_pack_bits (BatchCoder.pack_bits, the gatherer's payload) == the torch
    reference packing pack_bitstreams of the same streams: header of bit counts, then
    each stream's bytes back to back; ragged lengths, and a job of empty streams."""
    from lac_amd.batch import BatchCoder
    from lac_amd.dist import pack_bitstreams, unpack_bitstreams
    V, B, T = 1000, 777, 9
    coder = BatchCoder(V, B, prec=48, capacity_bits=T * 50 + 256, device=nccl_world1)
    bits, nbits, _, _ = _job(coder, 21, T, B, V)
    want, wlen = pack_bitstreams(bits, nbits, hdr)
    out = torch.full((B * (hdr + coder.bits_stride()) + 1,), 0xAB, dtype=torch.uint8, device=nccl_world1)
    ln = torch.zeros(1, dtype=torch.int64, device=nccl_world1)
    coder.pack_bits(out, hdr, ln)
    n = int(wlen)
    assert int(ln) == n and torch.equal(out[:n], want[:n])
    ub, un = unpack_bitstreams(out[:n], B, coder.bits_stride(), hdr)
    assert torch.equal(un, nbits)
    # no streams coded: every count 0, only the header
    coder.reset()
    coder.finish()
    coder.pack_bits(out, hdr, ln)
    assert int(ln) == B * hdr
    coder.close()
