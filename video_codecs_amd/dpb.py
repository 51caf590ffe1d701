"""The writer rank's shared decoded-picture buffer.

The multi-GPU path shards closed GOP segments across ranks (bench.closed_main, gop.ClosedSegments):
every rank encodes its own segments -- disjoint frame indices -- with references its own loop made
(hvx_hm_finish_picture + SAO on the device), so no reference picture and no decision input crosses
xGMI.  What does cross is each finished picture: after a picture's deblocking and SAO
(TEncGOP.cpp:1465, :1500) the rank's finished reconstructions of that POC (all its segments, the
planes as TComPicYuv holds them before extension, Y | Cb | Cr per segment) are gathered to rank 0
with ONE torch.distributed gather (RCCL over xGMI on the GPUs; gloo in the CPU tests) -- the shared
DPB the writer rank outputs from.  It is the only data-path collective of the path.  The gather is
asynchronous and the buffers are double-buffered, so picture t+1 decides while picture t moves; a
buffer is handed out again only after the gather that read it has completed.  Rank 0 keeps one
buffer per rank.
"""


class DpbGather:
    def __init__(self, world, rank, plane_shape, device, nbuf=2):
        import torch
        self.world, self.rank, self.nbuf, self.k = world, rank, nbuf, 0
        self.recon = [torch.zeros(plane_shape, dtype=torch.uint8, device=device) for _ in range(nbuf)]
        self.dpb = None
        if world > 1 and rank == 0:
            self.dpb = [[torch.zeros(plane_shape, dtype=torch.uint8, device=device) for _ in range(world)]
                        for _ in range(nbuf)]
        self.pending = [None] * nbuf

    def buffer(self):
        """The output buffer of the current picture (waits for the gather that last read it)."""
        b = self.k % self.nbuf
        if self.pending[b] is not None:
            self.pending[b].wait()
            self.pending[b] = None
        return self.recon[b]

    def send(self):
        """Gather the current picture's finished planes to rank 0 (no-op on one rank) and advance; returns its buffer index."""
        import torch.distributed as dist
        b = self.k % self.nbuf
        if self.world > 1 and dist.get_backend() == "gloo" and self.recon[b].is_cuda:
            # gloo gathers host tensors only (the rehearsal of several ranks on one GPU): staged, synchronous
            got = [self.recon[b].new_empty(self.recon[b].shape, device="cpu") for _ in range(self.world)] \
                if self.rank == 0 else None
            dist.gather(self.recon[b].cpu(), got, dst=0)
            if self.rank == 0:
                for r in range(self.world):
                    self.dpb[b][r].copy_(got[r])
        elif self.world > 1:
            self.pending[b] = dist.gather(self.recon[b], self.dpb[b] if self.rank == 0 else None, dst=0,
                                          async_op=True)
        self.k += 1
        return b

    def drain(self):
        """Wait for every outstanding gather."""
        for b in range(self.nbuf):
            if self.pending[b] is not None:
                self.pending[b].wait()
                self.pending[b] = None

    def last(self):
        """(own reconstruction, rank 0's gathered planes or None) of the latest sent picture."""
        b = (self.k - 1) % self.nbuf
        return self.recon[b], (self.dpb[b] if self.dpb is not None else None)
