"""The RCCL branch of the bitstream exchange (lac_amd/dist.py) on
the GPU, with a real BatchCoder: a one-rank nccl group (RCCL refuses two ranks
on one GPU -- "Duplicate GPU detected", tools/nccl_probe.py -- and the pool's
boxes have one MI355X).  Under nccl the root's own share is a P2P send to
itself in the same batch as every other rank's, so this runs every line of the
nccl path: packing into batched outboxes with device-chained offsets and lengths
in device-mapped host words, the sizes over the host (gloo), the side stream,
batch_isend_irecv, and outbox reuse at depth 2 and 3.
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


@pytest.mark.parametrize("batch,depth,jobs", [(1, 2, 5), (2, 2, 7), (3, 3, 11), (8, 2, 5)])
def test_rccl_gatherer_world1_real_coder(nccl_world1, batch, depth, jobs):
    from lac_amd.batch import BatchCoder
    from lac_amd.dist import BitstreamGatherer
    V, B, T = 1000, 96, 10
    coder = BatchCoder(V, B, prec=48, capacity_bits=T * 50 + 256, device=nccl_world1)
    g = BitstreamGatherer(coder, batch=batch, depth=depth)
    assert not g.gloo and g.self_p2p and g.native
    made, seen, when = [], [], []

    def record():
        for j in g.finished_jobs:
            if not seen or j > seen[-1][0]:
                b, n = g.last_unpacked(j)
                seen.append((j, b.clone(), n.clone()))
    for j in range(jobs):
        bits, nbits, _, _ = _job(coder, j, T, B, V)
        made.append((bits, nbits))
        g.submit()                                   # the next job's encode is enqueued behind it
        record()
        when.append(g.last_job)
    g.drain()
    record()
    # the coder shows its last job's output again after drain (its slot)
    assert torch.equal(coder.nbits_tensor(), made[-1][1]) and torch.equal(coder.bits_tensor(), made[-1][0])
    # and jobs after a drain continue the rotation
    for j in range(jobs, jobs + batch + 1):
        bits, nbits, _, _ = _job(coder, j, T, B, V)
        made.append((bits, nbits))
        g.submit()
        record()
    g.drain()
    record()
    assert [s[0] for s in seen] == list(range(1, jobs + batch + 2))
    for k, last in enumerate(when, start=1):     # the box of job k + 1 is prepared after job k
        assert last == max(0, k // batch - depth + 1) * batch, (k, last)
    for j, b, n in seen:
        want_b, want_n = made[j - 1]
        assert torch.equal(n, want_n)
        nb = ((want_n + 7) // 8).tolist()
        for r in range(B):
            assert torch.equal(b[r, :nb[r]], want_b[r, :nb[r]]) and not b[r, nb[r]:].any()
    assert g.jobs == jobs + batch + 1 and g.payload_bytes > 0
    g.close()
    coder.close()


def test_pack_bits_at_chains_jobs(nccl_world1):
    """lac_pack_bits_at appends jobs back to back through device-held offsets and writes
    each length into device-mapped host words (lac_host_alloc); a job that does not
    fit writes nothing and reports UINT64_MAX."""
    from lac_amd.batch import BatchCoder
    from lac_amd.dist import HostWords, pack_bitstreams
    V, B, T = 1000, 77, 6
    coder = BatchCoder(V, B, prec=48, capacity_bits=T * 50 + 256, device=nccl_world1)
    words = HostWords(coder.lib, 4)
    ends = torch.zeros(4, dtype=torch.int64, device=nccl_world1)
    cap = 3 * B * (2 + coder.bits_stride())
    out = torch.full((cap,), 0xCD, dtype=torch.uint8, device=nccl_world1)
    want = []
    for k in range(3):
        bits, nbits, _, _ = _job(coder, 40 + k, T, B, V)
        p, L = pack_bitstreams(bits, nbits, 2)
        want.append(p[:int(L)].clone())
        coder.pack_bits_at(out, 2, None if k == 0 else ends[k - 1:k], ends[k:k + 1], words.dev_addr(k))
    torch.cuda.synchronize()
    lens = [words[k] for k in range(3)]
    assert lens == [w.numel() for w in want]
    assert ends[:3].tolist() == [sum(lens[:k + 1]) for k in range(3)]
    assert torch.equal(out[:sum(lens)], torch.cat(want))
    small = torch.zeros(10, dtype=torch.uint8, device=nccl_world1)
    coder.pack_bits_at(small, 2, None, ends[3:4], words.dev_addr(3))
    torch.cuda.synchronize()
    assert words[3] == (1 << 64) - 1 and int(ends[3]) == 0 and not small.any()
    words.close()
    coder.close()


@pytest.mark.parametrize("streams", [77, 2500])
def test_pack_jobs_one_launch_equals_chained(nccl_world1, streams):
    """lac_pack_jobs packs several jobs' planes (strided rows, as the gatherer's slots) in
    one launch: bytes and ends equal packing them one by one; a base offset shifts
    everything; lengths land in the mapped host words."""
    import ctypes as C
    from lac_amd.batch import BatchCoder
    from lac_amd.dist import HostWords, pack_bitstreams
    from lac_amd._lib import check
    V, B, T, J = 1000, streams, 5, 3
    coder = BatchCoder(V, B, prec=48, capacity_bits=T * 50 + 256, device=nccl_world1)
    words = coder.output_words()
    planes = torch.zeros((J, words), dtype=torch.int64, device=nccl_world1)
    nbits = torch.zeros((J, B), dtype=torch.int64, device=nccl_world1)
    want = []
    for j in range(J):
        coder.set_output(planes[j], nbits[j])
        bits, nb, _, _ = _job(coder, 60 + j, T, B, V)
        p, L = pack_bitstreams(bits, nb, 2)
        want.append(p[:int(L)].clone())
    coder.set_output(None, None)
    host = HostWords(coder.lib, J)
    ends = torch.zeros(J, dtype=torch.int64, device=nccl_world1)
    base = torch.tensor([13], dtype=torch.int64, device=nccl_world1)
    cap = 13 + J * B * (2 + coder.bits_stride())
    out = torch.zeros(cap, dtype=torch.uint8, device=nccl_world1)
    check(coder.lib.lac_pack_jobs(0, C.c_void_p(planes.data_ptr()), words, C.c_void_p(nbits.data_ptr()), J, B,
                                  coder.bits_stride() // 8, C.c_void_p(out.data_ptr()), cap, 2,
                                  C.c_void_p(base.data_ptr()), C.c_void_p(ends.data_ptr()),
                                  C.c_void_p(host.dev_addr(0)), None))
    torch.cuda.synchronize()
    lens = [w.numel() for w in want]
    assert [host[j] for j in range(J)] == lens
    assert ends.tolist() == [13 + sum(lens[:j + 1]) for j in range(J)]
    assert not out[:13].any() and torch.equal(out[13:13 + sum(lens)], torch.cat(want))
    host.close()
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


def test_set_output_only_between_jobs():
    """lac_set_output refuses a redirect while streams hold unfinished coded symbols (their
    plane words are split between buffers: the finish would carry-add over the new ones)
    and while decoding; between jobs it redirects, and a redirect back to the buffers of
    the last finished job shows that job again (lac_pack_bits packs it)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from lac_amd.batch import BatchCoder
    from lac_amd._lib import LacError, LAC_E_STATE
    from lac_amd.dist import pack_bitstreams
    from lac_amd import synth
    dev = torch.device("cuda", 0)
    V, B, T = 1000, 40, 8
    coder = BatchCoder(V, B, prec=48, capacity_bits=T * 50 + 256, device=dev)
    words = coder.output_words()
    planes = torch.zeros((2, words), dtype=torch.int64, device=dev)
    nbits = torch.zeros((2, B), dtype=torch.int64, device=dev)
    pmf, sym = synth.make_batch(77, T, B, V, "loguniform")
    dpmf, dsym = torch.from_numpy(pmf.view(np.int32)).to(dev), torch.from_numpy(sym).to(dev)
    coder.set_output(planes[0], nbits[0])                   # fresh context: allowed
    coder.reset()
    coder.encode(dpmf[:T // 2], dsym[:T // 2])              # an open encode ...
    with pytest.raises(LacError) as e:
        coder.set_output(planes[1], nbits[1])
    assert e.value.code == LAC_E_STATE
    coder.encode(dpmf[T // 2:], dsym[T // 2:])
    coder.finish()                                          # ... finished: the bytes are whole
    want_b, want_n = coder.bits_tensor().clone(), coder.nbits_tensor().clone()
    ref = BatchCoder(V, B, prec=48, capacity_bits=T * 50 + 256, device=dev)
    ref.encode_job(dpmf, dsym)
    # (each stream's ceil(nbits/8) bytes: past them a fresh context's words hold whatever the
    # buffer held before)
    live = torch.arange(want_b.shape[1], device=dev)[None, :] < ((want_n + 7) // 8)[:, None]
    assert torch.equal(want_n, ref.nbits_tensor())
    assert torch.equal(torch.where(live, want_b, 0), torch.where(live, ref.bits_tensor(), 0))
    coder.set_output(planes[1], nbits[1])                   # between jobs
    coder.encode_job(dpmf, dsym)
    assert torch.equal(coder.nbits_tensor(), want_n)
    coder.set_output(planes[0], nbits[0])                   # the previous job's buffers: not finished
    out = torch.zeros(B * (2 + coder.bits_stride()) + 1, dtype=torch.uint8, device=dev)
    ln = torch.zeros(1, dtype=torch.int64, device=dev)
    with pytest.raises(LacError):
        coder.pack_bits(out, 2, ln)
    coder.set_output(planes[1], nbits[1])                   # the last finished job's: packs again
    coder.pack_bits(out, 2, ln)
    p, L = pack_bitstreams(want_b, want_n, 2)
    assert int(ln) == int(L) and torch.equal(out[:int(L)], p[:int(L)])
    coder.decode_open()                                     # decoding: refused
    with pytest.raises(LacError) as e:
        coder.set_output(None, None)
    assert e.value.code == LAC_E_STATE
    coder.reset()
    coder.set_output(None, None)
    ref.close()
    coder.close()
