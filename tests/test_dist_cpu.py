"""The multi-rank path of bench.py on CPU: world_size-2 torch.distributed over gloo.

bench.py shards independent pictures across ranks: each rank decides its own
pictures, the timed region is bracketed by barriers on every rank, the time is the MAX over ranks
and the value counts the units of ALL ranks.  Here the per-rank step is the CPU restatement of the
HM-exact decision (oracle/hvx_oracle_cu.c) on small pictures, so the orchestration (picture
assignment, barrier + max-over-ranks timing, aggregation, DPB gather) is tested without a GPU.
The gloo rendezvous uses 127.0.0.1.
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


def test_segment_and_aggregate_contract():
    import bench
    plans = [bench.HmPlan(3840, 2160, 62, 4, 32, 1, r) for r in range(8)]
    flat = [f for p in plans for f in p.frames()]
    assert len(flat) == len(set(flat)) == 8 * 66  # 8 ranks, disjoint synthetic frame ranges
    assert bench.aggregate(2040, 10, 8, 2.0) == 2040 * 10 * 8 / 2.0
    assert bench.b_ctu(4) == 6144 * 6 + 2 * 6144 + 16 * 256 == 53248  # SURVEY 8(d), LDP 4 refs


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


# ---- config 5: closed GOP segments per rank (bench.closed_main), decided by the restatement ----
CW, CH, CSEGS, CSTEP = 128, 64, 2, 1  # 2 segments of 128x64 per rank, 1 CTU per chain per step


def _closed_args(warmup, steps):
    import argparse
    return argparse.Namespace(segs=CSEGS, closed_ctus=CSTEP, warmup=warmup, steps=steps, qp=32)


def _closed_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from tests.segment_port import PortSegments
    gathered = []
    work, elapsed, sec, ctus, byt, dpb_ok, n_gathered = bench.closed_main(
        _closed_args(2, 4), rank, world, device="cpu", segments_cls=PortSegments, size=(CW, CH))
    # every finished picture of the rank's segments, in the order they were gathered
    own = np.stack([np.concatenate([np.concatenate([p.numpy().reshape(-1) for p in r["rec"]]) for r in res])
                    for res in work.cs.finished_log])
    np.save(os.path.join(outdir, f"own{rank}.npy"), own)
    if rank == 0:
        np.save(os.path.join(outdir, "dpb_last.npy"), np.stack([t.numpy() for t in work.dpb.last()[1]]))
    parts = np.stack([np.stack([r["parts"] for r in res]) for res in work.cs.finished_log])
    np.save(os.path.join(outdir, f"parts{rank}.npy"), parts)
    seeds = [bench.closed_seed(rank, CSEGS, s, g.poc) for s in range(CSEGS) for g in work.plan]
    np.save(os.path.join(outdir, f"meta{rank}.npy"), np.array([elapsed, ctus, n_gathered, int(bool(dpb_ok))] + seeds,
                                                               np.float64))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_closed_segments_gloo(tmp_path):
    """BASELINE config 5's multi-GPU path (bench.closed_main) on two ranks over gloo, with the
    restatement standing in for the device (tests/segment_port.py): each rank encodes its OWN closed LDP
    segments (frame indices disjoint across ranks: bench.closed_seed), every P picture decided against
    the references its own loop made; after every picture each segment's finished (deblocked) picture is
    gathered to rank 0.  Checks: the same max-over-ranks time on both ranks; the timed CTUs = K steps of
    every chain; the two ranks' pictures differ; rank 0's DPB holds each rank's finished pictures
    bit-exactly; and each rank's decisions equal a single-process run of its segments."""
    import torch.multiprocessing as tmp
    import bench
    from tests.segment_port import PortSegments
    world = 2
    tmp.spawn(_closed_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    metas = [np.load(tmp_path / f"meta{r}.npy") for r in range(world)]
    assert metas[0][0] == metas[1][0]  # max over ranks
    assert int(metas[0][1]) == CSEGS * 1 * CSTEP * 4  # one chain per 128x64 picture, 4 timed steps
    assert all(int(m[3]) == 1 for m in metas[:1])  # rank 0's own slot of the gather equals its buffer
    assert not set(metas[0][4:]) & set(metas[1][4:])  # disjoint synthetic frames
    owns = [np.load(tmp_path / f"own{r}.npy") for r in range(world)]
    assert owns[0].shape == owns[1].shape and int(metas[0][2]) == owns[0].shape[0] == 3  # I, P, P finished
    assert not np.array_equal(owns[0], owns[1])
    last = np.load(tmp_path / "dpb_last.npy")  # rank 0's DPB after the last gather: every rank's last picture
    for r in range(world):
        np.testing.assert_array_equal(last[r], owns[r][-1])
    # a single-process run of rank 1's segments decides the same CTUs and makes the same pictures
    work, *_ = bench.closed_main(_closed_args(2, 4), 1, 1, device="cpu", segments_cls=PortSegments, size=(CW, CH))
    parts1 = np.load(tmp_path / "parts1.npy")
    np.testing.assert_array_equal(np.stack([np.stack([r["parts"] for r in res]) for res in work.cs.finished_log]), parts1)


def test_closed_port_segment_vs_hm():
    """The closed-segment orchestration (gop.ClosedSegments' picture set-up, reference lists, DPB and
    collocated-field bookkeeping) with the restatement deciding: HM's own closed LDP encode (I, P, P,
    416x240, SAO off, one slice per picture: tests/golden/ctu_ldp_nosao.bin) is reproduced CTU for CTU,
    every P picture decided against the references this loop made."""
    from tests import golden_cases as gc
    from tests import hm_cases
    from tests.segment_port import PortSegments
    from video_codecs_amd import gop
    g = gc.load("ctu_ldp_nosao.bin")
    psz = 416 * 240 * 3 // 2
    plan = gop.load_plan("ldp", 3)
    cs = PortSegments(plan, 416, 240, [27], lambda s, poc: hm_cases.yuv_split(g["org"][poc * psz:(poc + 1) * psz], 416, 240),
                      rows=4, threads=4)
    while cs.t < 3:
        cs.step()
    for pic, res in enumerate(cs.finished_log):
        first, n = int(g["pic_i32"][pic][hm_cases.P_FIRST_CTU]), int(g["pic_i32"][pic][hm_cases.P_NCTU])
        np.testing.assert_array_equal(res[0]["parts"], g["ctu_parts"][first:first + n], err_msg=f"pic {pic}")
