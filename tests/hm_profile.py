"""Debugging aid: per-category cycle profile of the HM engine (an HM_PROFILE build of libhvx,
selected with HVX_LIB_PATH) on the captured pictures.  python -m tests.hm_profile [mode] [capture]"""
import sys
import time

import numpy as np

from tests import hm_cases

NAMES = ["ME", "MC", "TPL", "TUF", "TUI", "COEF", "EST", "IFP", "IPRED", "DIST", "CTU", "ENC", "TUF4", "TUF8", "TUF16", "TUF32",
         "C.desc", "C.stage", "C.walk", "T.in", "T.fwd", "T.out", "xform", "rdoq", "COEF4", "COEF8", "COEF16", "COEF32",
         "rdoqA", "rdoqB", "rdoqC", "rdoqDE"]
NPROF = 32

def report(prof, n, head):
    prof = prof.astype(np.float64)
    print(head)
    tot, calls = prof[:, 0, :].sum(0), prof[:, 1, :].sum(0)
    ctu = tot[10]
    for i, nm in enumerate(NAMES):
        if calls[i]:
            print("  %-6s %14.0f ticks %8.1f%% of CTU  calls %9d  ticks/call %10.0f  calls/CTU %8.1f" % (
                nm, tot[i], 100 * tot[i] / ctu, calls[i], tot[i] / calls[i], calls[i] / n))
    per_job = prof[:, 0, 10]
    print("  CTU ticks per job: min %.3g med %.3g max %.3g" % (per_job.min(), np.median(per_job), per_job.max()))


def bench_profile(pics, steps):
    """The bench workload (bench.HmWorkload, 2160p random) with `pics` pictures for `steps` steps."""
    import torch
    import bench
    from video_codecs_amd import hvx
    hvx.context()
    w = bench.HmWorkload(3840, 2160, pics, 4, 32, 1, 0)
    rec = torch.zeros(w.slots * 6144, dtype=torch.uint8, device="cuda")
    for s in range(steps):
        torch.cuda.synchronize()
        t0 = time.time()
        w.step(rec)
        torch.cuda.synchronize()
        dt = time.time() - t0
        sb = w.eng.reserve(w.n_jobs)
        # State.status[4] | dbg[4] | prof[2][32] (csrc/hvx_hm.hpp)
        st = w.eng.state[:w.n_jobs * sb].view(w.n_jobs, sb)[:, :32 + 16 * NPROF].cpu().numpy().copy()
        prof = st[:, 32:32 + 16 * NPROF].copy().view(np.uint64).reshape(w.n_jobs, 2, NPROF)
        report(prof, w.n_jobs, "bench step %d: %d chains, %.3f s" % (s, w.n_jobs, dt))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "bench":
        bench_profile(int(sys.argv[2]), int(sys.argv[3]))
        sys.exit(0)
    mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    name = sys.argv[2] if len(sys.argv) > 2 else "ctu_ldp_smooth.bin"
    pics = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else None
    hm_cases.run_capture(name, mode, pics)  # warm-up (module load)
    t0 = time.time()
    g, plan, out = hm_cases.run_capture(name, mode, pics)
    dt = time.time() - t0
    bad = hm_cases.compare(g, plan, out)
    prof = hm_cases.LAST_ENGINE[0].last_prof.astype(np.float64)
    n = sum(p[2] for p in plan)
    print("%s mode %d: %d CTUs, %d mismatches, host wall %.2f s" % (name, mode, n, len(bad), dt))
    tot, calls = prof[:, 0, :].sum(0), prof[:, 1, :].sum(0)
    ctu = tot[10]
    for i, nm in enumerate(NAMES):
        if calls[i]:
            print("  %-6s %14.0f ticks %8.1f%% of CTU  calls %9d  ticks/call %10.0f" % (nm, tot[i], 100 * tot[i] / ctu, calls[i], tot[i] / calls[i]))
    per_job = prof[:, 0, 10]
    print("  CTU ticks per job: min %.3g med %.3g max %.3g" % (per_job.min(), np.median(per_job), per_job.max()))
