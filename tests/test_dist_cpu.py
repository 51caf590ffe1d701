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


# ---- closed GOP segments per rank (config 5's unit), decided by the restatement ----
def _closed_segment(g, rank):
    """The LDP segment of tests/golden/ctu_ldp_nosao.bin (I, P, P; SAO off) decided in closed loop by
    the restatement: every picture from the capture's original and slice-start states only, each P
    picture against the reference pictures this loop made (restatement decisions -> boundary
    strengths -> oracle loopFilterPic), never the capture's.  Returns [(poc, parts, recon planes,
    reference planes)]."""
    import oracle
    from oracle import hm_ctu
    from tests import hm_cases
    from video_codecs_amd import _abi
    made = {}
    out = []
    gl = dict(g)
    refpoc = [int(p) for p in g["refpic_poc"]]
    for pic, pi in enumerate(g["pic_i32"]):
        poc, w, h = int(pi[hm_cases.P_POC]), int(pi[hm_cases.P_W]), int(pi[hm_cases.P_H])
        first, n = int(pi[hm_cases.P_FIRST_CTU]), int(pi[hm_cases.P_NCTU])
        psz = w * h * 3 // 2
        # the references this loop made, in the capture's reference-plane slots
        rp = np.array(g["refpic"], copy=True)
        for k, q in enumerate(refpoc):
            if q in made:
                rp[k * psz:(k + 1) * psz] = np.concatenate([p.reshape(-1) for p in made[q]])
            elif q < poc:
                raise AssertionError("reference POC %d not made yet" % q)
        gl["refpic"] = rp
        r = hm_ctu.replay(gl, pic, mode=1)
        rec = [np.zeros((h >> (1 if c else 0), w >> (1 if c else 0)), np.uint8) for c in range(3)]
        wc = (w + 63) // 64
        for a in range(n):
            ax, ay = a % wc, a // wc
            t = r["recon"][a]
            yy, xx = min(64, h - ay * 64), min(64, w - ax * 64)
            rec[0][ay * 64:ay * 64 + yy, ax * 64:ax * 64 + xx] = t[:4096].reshape(64, 64)[:yy, :xx]
            for c in (1, 2):
                cpl = t[4096 + (c - 1) * 1024:4096 + c * 1024].reshape(32, 32)
                rec[c][ay * 32:ay * 32 + yy // 2, ax * 32:ax * 32 + xx // 2] = cpl[:yy // 2, :xx // 2]
        rpoc = np.array([pi[hm_cases.P_REFPOC0:hm_cases.P_REFPOC0 + 4], pi[hm_cases.P_REFPOC1:hm_cases.P_REFPOC1 + 4]])
        bv, bh, qp = hm_ctu.boundary_strength(w, h, r["parts"], rpoc, int(pi[hm_cases.P_SLICE_TYPE]) == 0)
        ref = oracle.deblock(*rec, bv.reshape(-1), bh.reshape(-1), qp.reshape(-1), _abi.deblock_params(w, h))
        made[poc] = ref
        out.append((poc, r["parts"], rec, ref))
    return out


def _closed_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests import golden_cases as gc
    from video_codecs_amd.dpb import DpbGather
    g = gc.load("ctu_ldp_nosao.bin")
    w, h = int(g["pic_i32"][0][0]), int(g["pic_i32"][0][1])
    seg = _closed_segment(g, rank)
    # every finished reference picture of the rank's segment goes to rank 0's DPB
    dpb = DpbGather(world, rank, (w * h * 3 // 2,), "cpu")
    got = []
    for poc, _, _, ref in seg:
        buf = dpb.buffer()
        buf.copy_(torch.from_numpy(np.concatenate([p.reshape(-1) for p in ref])))
        b = dpb.send()
        dpb.drain()
        if rank == 0:
            got.append(np.stack([t.numpy().copy() for t in dpb.dpb[b]]))
    np.save(os.path.join(outdir, f"closed_parts{rank}.npy"), np.stack([s[1] for s in seg]))
    if rank == 0:
        np.save(os.path.join(outdir, "closed_dpb.npy"), np.stack(got))
        np.save(os.path.join(outdir, "closed_refs0.npy"),
                np.stack([np.concatenate([p.reshape(-1) for p in s[3]]) for s in seg]))
    dist.destroy_process_group()


def test_two_rank_closed_segments_gloo(tmp_path):
    """Config 5's unit on two ranks (gloo): each rank encodes a closed LDP segment (I, P, P) with the
    restatement -- every P picture decided against the reference pictures its own loop made (the
    restatement's decisions, boundary strengths and loopFilterPic), not the capture's -- and every
    picture equals HM's own decisions (tests/golden/ctu_ldp_nosao.bin, SAO off); every finished
    reference picture goes to rank 0 through DpbGather, where each rank's copy equals that rank's."""
    import torch.multiprocessing as tmp
    from tests import golden_cases as gc
    from tests import hm_cases
    world = 2
    tmp.spawn(_closed_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    g = gc.load("ctu_ldp_nosao.bin")
    for r in range(world):
        parts = np.load(tmp_path / f"closed_parts{r}.npy")
        for pic, pi in enumerate(g["pic_i32"]):
            first, n = int(pi[hm_cases.P_FIRST_CTU]), int(pi[hm_cases.P_NCTU])
            np.testing.assert_array_equal(parts[pic], g["ctu_parts"][first:first + n], err_msg=f"rank {r} pic {pic}")
    dpb, refs0 = np.load(tmp_path / "closed_dpb.npy"), np.load(tmp_path / "closed_refs0.npy")
    assert dpb.shape[:2] == (3, world)
    for k in range(3):
        for r in range(world):
            np.testing.assert_array_equal(dpb[k, r], refs0[k])  # the same segment on both ranks here
    # the made references equal HM's reference pictures
    psz = refs0.shape[1]
    for k, q in enumerate(int(p) for p in g["refpic_poc"]):
        np.testing.assert_array_equal(refs0[q], g["refpic"][k * psz:(k + 1) * psz])


def test_closed_loop_geometry_and_jobs():
    """bench.closed_loop_measure's slicing (CPU): at 1088p one chain per CTU row; at 2160p two rows
    per slice, the partial bottom row inside the last slice (a one-row slicing is refused); every
    launch's jobs advance every chain by the same CTUs, and the launches of a picture cover each
    slice's CTUs exactly once, resumed after the first."""
    import bench
    assert bench.closed_loop_geometry(1920, 1088, 1, 6) == (30, 17, 17, 30)
    assert bench.closed_loop_geometry(3840, 2160, 2, 8) == (60, 34, 17, 120)
    with pytest.raises(AssertionError):
        bench.closed_loop_geometry(3840, 2160, 1, 6)
    wc, hc, nch, cl = bench.closed_loop_geometry(3840, 2160, 2, 8)
    seen = {}
    for L in range(cl // 8):
        for seg, first, n, s0, s1, resume in bench.closed_loop_specs(3, nch, cl, L, 8):
            assert s0 <= first and first + n - 1 <= s1 and s1 - s0 + 1 == cl and resume == (L > 0)
            for a in range(first, first + n):
                seen[(seg, a)] = seen.get((seg, a), 0) + 1
    assert sorted(seen) == [(s, a) for s in range(3) for a in range(wc * hc)] and set(seen.values()) == {1}
    # encoder_lowdelay_P_main.cfg:24-27 (Frame1..4: QP offset, QPFactor)
    assert [bench.LDP_GOP[k][:2] for k in (1, 2, 3, 4)] == [(3, 0.4624), (2, 0.4624), (3, 0.4624), (1, 0.578)]
