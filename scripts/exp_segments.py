"""Experiment: K independent segments encoded concurrently on one GPU (private hvx_ctx + torch
stream per segment).  Prints ms per step (K pictures) and aggregate CTUs/s for each K."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from video_codecs_amd import hvx, synth

W, H, nref, qp = int(os.environ.get("W", 3840)), int(os.environ.get("H", 2160)), 4, 32
steps = 8
res = {}
for K in (1, 2, 3, 4):
    segs = []
    for s in range(K):
        planes = [torch.from_numpy(synth.luma_plane(W, H, s * (nref + 1) + f)).cuda() for f in range(nref + 1)]
        ptrs = torch.tensor([hvx.plane_origin_ptr(t, W) for t in planes[:nref]], dtype=torch.int64).cuda()
        an = hvx.CtuAnalyzer(W, H, nref, qp, ctx=hvx.new_context())
        segs.append(dict(cur=planes[nref], refs=planes, ptrs=ptrs, an=an, st=torch.cuda.Stream(),
                         rec=torch.zeros_like(planes[nref]), ref=torch.zeros_like(planes[nref])))
    torch.cuda.synchronize()

    def step():
        for g in segs:
            with torch.cuda.stream(g["st"]):
                g["an"].encode(g["cur"], g["ptrs"], g["rec"], g["ref"])
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    # segment results equal a lone encode of the same picture
    ok = True
    for g in segs:
        d = g["an"].decisions().tobytes()
        a1 = hvx.CtuAnalyzer(W, H, nref, qp)
        r1 = torch.zeros_like(g["cur"])
        a1.encode(g["cur"], g["ptrs"], r1, None)
        torch.cuda.synchronize()
        ok &= a1.decisions().tobytes() == d and torch.equal(r1, g["rec"])
        del a1
    res[K] = {"ms_per_step": round(ms, 3), "ctus_per_s": round(K * segs[0]["an"].nctu / ms * 1e3, 1), "equal": bool(ok)}
    print(K, res[K], flush=True)
    del segs
    torch.cuda.empty_cache()
print(json.dumps(res))
