"""The multi-rank path of bench.py on CPU: world_size-2 torch.distributed over gloo.

bench.py shards the CTU analysis pass by independent GOP segments: each rank
analyses its own frames, the timed region is bracketed by barriers on every rank, the time
is the MAX over ranks and the value counts the units of ALL ranks.  Here the per-rank step is
the CPU restatement of the same pass (oracle/hvx_oracle.c) on a small picture, so the
orchestration (segment assignment, barrier + max-over-ranks timing, aggregation) is tested
without a GPU.  The gloo rendezvous uses 127.0.0.1.
"""
import os
import socket

import numpy as np
import pytest

W, H, NREF, QP, STEPS, WARMUP = 128, 64, 1, 32, 2, 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _analyze(planes):
    import oracle
    from video_codecs_amd import _abi
    params = _abi.ctu_params(W, H, NREF, QP)
    est = _abi.load_estbits_p_luma()
    ncx, ncy = (W + 63) // 64, (H + 63) // 64
    return np.stack([oracle.ctu_analyze(planes[NREF], planes[:NREF], params, est, c % ncx, c // ncx)
                     for c in range(ncx * ncy)])


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    frames = bench.segment_frames(rank, NREF)
    planes = [bench.luma_plane(W, H, f) for f in frames]
    box = {}

    def step():
        box["res"] = _analyze(planes)

    elapsed = bench.timed_steps(step, STEPS, WARMUP, world, "cpu", lambda: None)
    nctu = box["res"].shape[0]
    value = bench.aggregate(nctu, STEPS, world, elapsed)
    np.save(os.path.join(outdir, f"res{rank}.npy"), box["res"].view(np.uint8))
    np.save(os.path.join(outdir, f"meta{rank}.npy"), np.array([elapsed, value, nctu] + frames, dtype=np.float64))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_segments_gloo(tmp_path):
    import torch.multiprocessing as tmp
    world = 2
    tmp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    metas = [np.load(tmp_path / f"meta{r}.npy") for r in range(world)]
    res = [np.load(tmp_path / f"res{r}.npy") for r in range(world)]
    # max-over-ranks timing: every rank ends with the same elapsed and the same whole-job value
    assert metas[0][0] == metas[1][0]
    nctu = int(metas[0][2])
    assert metas[0][1] == pytest.approx(nctu * STEPS * world / metas[0][0])
    # disjoint segments: rank r analyses frames r*(nref+1) .. r*(nref+1)+nref
    f0, f1 = [int(x) for x in metas[0][3:]], [int(x) for x in metas[1][3:]]
    assert f0 == [0, 1] and f1 == [2, 3] and not set(f0) & set(f1)
    assert res[0].tobytes() != res[1].tobytes()
    # each rank's result is exactly the single-process result for its own segment
    import bench
    for r, frames in ((0, f0), (1, f1)):
        exp = _analyze([bench.luma_plane(W, H, f) for f in frames])
        assert res[r].tobytes() == exp.view(np.uint8).tobytes()


def test_segment_and_aggregate_contract():
    import bench
    segs = [bench.segment_frames(r, 4) for r in range(8)]
    flat = [f for s in segs for f in s]
    assert len(flat) == len(set(flat)) == 40  # 8 closed, disjoint segments of nref+1 frames
    assert bench.aggregate(2040, 10, 8, 2.0) == 2040 * 10 * 8 / 2.0
    assert bench.b_ctu(4) == 6144 * 6 + 2 * 6144 + 16 * 256 == 53248  # SURVEY 8(d), LDP 4 refs


def _decide_picture(planes, rec_flat):
    """The oracle's full 4:2:0 step (analysis + CU decision + reconstruction) into rec_flat (one
    Y | Cb | Cr picture buffer, the layout the bench step gathers)."""
    import oracle
    from video_codecs_amd import _abi, hvx
    params = _abi.ctu_params(W, H, NREF, QP, chroma=True)
    est7 = _abi.estbits_p_yuv(oracle.estbits_update)
    st, eb = _abi.load_ctx_p_states(), _abi.load_entropy_bits()
    rec = hvx.yuv_views(rec_flat, W, H)
    refs = planes[:NREF]
    refs3 = ([r[0] for r in refs], [r[1] for r in refs], [r[2] for r in refs])
    ncx, ncy = (W + 63) // 64, (H + 63) // 64
    for c in range(ncx * ncy):
        oracle.ctu_decide_yuv(planes[NREF], refs3, params, est7, st, eb, c % ncx, c // ncx, rec)


def _dpb_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from video_codecs_amd.dpb import DpbGather
    from video_codecs_amd import hvx
    planes = [bench.yuv_planes(W, H, f) for f in bench.segment_frames(rank, NREF)]
    g = DpbGather(world, rank, (hvx.yuv_bytes(W, H),), "cpu")

    def step():  # the bench step's shape: decide into the DPB buffer, then the async gather
        _decide_picture(planes, g.buffer().numpy())
        g.send()

    elapsed = bench.timed_steps(step, STEPS, WARMUP, world, "cpu", g.drain)
    own, gathered = g.last()
    np.save(os.path.join(outdir, f"own{rank}.npy"), own.numpy())
    if rank == 0:
        np.save(os.path.join(outdir, "dpb.npy"), np.stack([t.numpy() for t in gathered]))
    np.save(os.path.join(outdir, f"t{rank}.npy"), np.array([elapsed, g.k]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_dpb_gather_gloo(tmp_path):
    # the per-picture DPB gather: after STEPS + WARMUP pictures through two
    # alternating buffers, rank 0 holds each rank's latest 4:2:0 reconstruction (one Y | Cb | Cr
    # buffer per picture), and that reconstruction is exactly the single-process one of the rank's
    # own segment
    import torch.multiprocessing as tmp
    world = 2
    tmp.spawn(_dpb_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    dpb = np.load(tmp_path / "dpb.npy")
    assert dpb.shape[0] == world
    import bench
    for r in range(world):
        own = np.load(tmp_path / f"own{r}.npy")
        np.testing.assert_array_equal(dpb[r], own)
        exp = np.zeros_like(own)
        _decide_picture([bench.yuv_planes(W, H, f) for f in bench.segment_frames(r, NREF)], exp)
        np.testing.assert_array_equal(own, exp)
        assert int(np.load(tmp_path / f"t{r}.npy")[1]) == STEPS + WARMUP
    assert not np.array_equal(dpb[0], dpb[1])


# ---- the headline's orchestration (bench.HmPlan / HmWorkload) with the HM-exact restatement ----
HW, HH, HPICS, HNREF = 128, 112, 2, 2  # 2 x 2 CTUs: one chain per picture over both row slices


def _hm_step(plan):
    """One bench step with every chain run to its end on the CPU restatement (hvxo_hm_chains): the
    reconstructed CTUs of every picture's chains in the bench's DPB slot order (chain k of picture
    p -> slots (p * rows + k) * per_chain ...)."""
    from oracle import hm_ctu
    per_chain = plan.wc * (2 if plan.merge_last else 1)
    out = np.zeros((plan.n_jobs * per_chain, 6144), np.uint8)
    for p in range(plan.pics):
        pi, pf, org, refs, col = plan.host_inputs(p)
        first = np.arange(plan.rows, dtype=np.int32) * plan.wc
        r = hm_ctu.chains(pi, pf, org, refs, plan.entry, first, per_chain, plan.wc, threads=1, col_field=col)
        out[p * plan.rows * per_chain:(p + 1) * plan.rows * per_chain] = r["recon"]
    return out


def _hm_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from video_codecs_amd.dpb import DpbGather
    plan = bench.HmPlan(HW, HH, HPICS, HNREF, QP, (HW + 63) // 64, rank)
    per_chain = plan.wc * (2 if plan.merge_last else 1)
    g = DpbGather(world, rank, (plan.n_jobs * per_chain * 6144,), "cpu")

    def step():  # bench.main's step: decide into the DPB buffer, then the asynchronous gather
        g.buffer().numpy()[:] = _hm_step(plan).reshape(-1)
        g.send()

    elapsed = bench.timed_steps(step, STEPS - 1, WARMUP, world, "cpu", g.drain)
    units = plan.n_jobs * per_chain
    value = bench.aggregate(units, STEPS - 1, world, elapsed)
    own, gathered = g.last()
    np.save(os.path.join(outdir, f"own{rank}.npy"), own.numpy())
    if rank == 0:
        np.save(os.path.join(outdir, "dpb.npy"), np.stack([t.numpy() for t in gathered]))
    np.save(os.path.join(outdir, f"meta{rank}.npy"), np.array([elapsed, value, units, g.k] + plan.frames(), np.float64))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_hm_workload_gloo(tmp_path):
    """bench.py's headline orchestration on two ranks (gloo): each rank decides its own pictures
    (disjoint synthetic frame ranges, HmPlan), chained across the partial bottom row's slice as the
    GPU chains are, through the HM-exact restatement; the per-step DPB gather leaves every rank's
    reconstructed CTUs on rank 0, identical to that rank's own buffer and to a single-process run of
    its plan; the timed region ends with the same max-over-ranks time on both ranks and the
    whole-job value counts the CTUs of both."""
    import torch.multiprocessing as tmp
    import bench
    world = 2
    tmp.spawn(_hm_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    metas = [np.load(tmp_path / f"meta{r}.npy") for r in range(world)]
    assert metas[0][0] == metas[1][0]  # max over ranks
    units = int(metas[0][2])
    assert units == HPICS * 4
    assert metas[0][1] == pytest.approx(units * (STEPS - 1) * world / metas[0][0])
    frames = [set(int(f) for f in m[4:]) for m in metas]
    assert len(frames[0]) == len(frames[1]) == HPICS + HNREF and not frames[0] & frames[1]
    dpb = np.load(tmp_path / "dpb.npy")
    for r in range(world):
        own = np.load(tmp_path / f"own{r}.npy")
        assert int(metas[r][3]) == STEPS  # pictures sent: warmup + timed
        np.testing.assert_array_equal(dpb[r], own)
        exp = _hm_step(bench.HmPlan(HW, HH, HPICS, HNREF, QP, (HW + 63) // 64, r))
        np.testing.assert_array_equal(own.reshape(-1, 6144), exp)
    assert not np.array_equal(dpb[0], dpb[1])
