"""Multi-GPU frame pipeline: one process per GPU; rank r renders the
interleaved row bands r, r+P, r+2P, ... of every frame into a local buffer, the buffers
are gathered to rank 0 with torch.distributed (RCCL over xGMI on MI355X, gloo in the CPU
tests) and rank 0 reassembles the frame. Frame k's gather overlaps frame k+1's render:
local buffers and gather targets alternate, and rank 0 unshuffles frame k only after
issuing frame k+1's render. With `inflight` F > 1, frames rotate over F streams and
F buffer sets, so frame k+1's render also overlaps frame k's: a rank's share of one
frame is short next to its longest pixel's sequential march.

The band renderer and the unshuffle are injected (libfrm on the GPU, the oracle/numpy in
tests) so the scheduling logic here is exactly what bench.py runs."""
import contextlib

import torch
import torch.distributed as dist

from . import tiling


class RowTiledFrame:
    def __init__(self, width, height, rank, world, band_rows, device, render_bands, unshuffle,
                 group=None, inflight=1, streams=None, collective=None, stage_host=None, batch=1):
        """render_bands(buf, band_rows, first_band, band_stride, slot, count): enqueue the
        render of this rank's bands of the next `count` frames (1 <= count <= batch) into the
        uint8 tensor buf (device memory for the GPU path), frame b at b * nbytes, for launch
        slot `slot` (k % inflight; the GPU path renders it on streams[slot]).
        unshuffle(gathered, frame, slot): rank 0 only; rank-major band buffers -> row-major
        frame. inflight = frames in flight: frame k's render, gather and unshuffle are
        enqueued on streams[k % inflight] (torch streams; None = the current stream, as in
        the CPU tests), so up to `inflight` frames overlap on the GPU. collective: gather
        through torch.distributed (default: when world > 1; True with world 1 runs the
        same gather/unshuffle path on one rank, a test hook for RCCL on one GPU).
        batch: frames per launch (frm_render_bands_batch): a launch renders up to `batch`
        frames (run(n) issues n // batch full launches and one launch of the remainder, so
        exactly n frames are rendered), one frame's bands each; one gather moves them all;
        unshuffle(gathered, rank_stride, frame, slot) rebuilds one frame from rank-major
        buffers rank_stride bytes apart.
        stage_host: gather through host copies of the band buffers (default: when the
        backend is gloo and the buffers live on a GPU). A test hook: RCCL refuses two ranks
        on one GPU, so a 1-GPU box runs the row split with gloo, whose gather takes host
        tensors only; the RCCL path never stages."""
        self.width, self.height = width, height
        self.rank, self.world = rank, world
        self.band_rows = band_rows
        self.render_bands = render_bands
        self.unshuffle = unshuffle
        self.group = group
        self.collective = world > 1 if collective is None else bool(collective)
        self.inflight = max(1, inflight)
        self.streams = streams
        if streams is not None and len(streams) != self.inflight:
            raise ValueError(f"{len(streams)} streams for {self.inflight} frames in flight")
        if stage_host is None:
            stage_host = (self.collective and torch.device(device).type == "cuda"
                          and dist.get_backend(group) == "gloo")
        self.stage_host = bool(stage_host)
        self.batch = max(1, batch)
        self.rows_local = tiling.rank_buffer_rows(height, band_rows, world)
        self.nbytes = self.rows_local * width * 4  # one frame's bands (padded)
        # buffer k % nbuf serves frame k. Reuse is safe in stream order: frame k + nbuf runs
        # on frame k's stream (nbuf is a multiple of inflight), after frame k's gather wait
        # and unshuffle, which _finish(k) enqueues before frame k + nbuf is issued.
        nbuf = self.inflight if self.inflight > 1 else (2 if self.collective else 1)
        self.nbuf = nbuf
        B = self.batch
        self.bufs = [torch.zeros(B * self.nbytes, dtype=torch.uint8, device=device) for _ in range(nbuf)]
        self.gathered = self.frames = None
        if self.collective and rank == 0:
            self.gathered = [torch.zeros(world * B * self.nbytes, dtype=torch.uint8, device=device)
                             for _ in range(nbuf)]
            self.frames = [torch.zeros(B * height * width * 4, dtype=torch.uint8, device=device)
                           for _ in range(nbuf)]
        self.frames_done = 0
        self.last = 0
        self.last_count = 1

    def _stream(self, k):
        if self.streams is None:
            return contextlib.nullcontext()
        return torch.cuda.stream(self.streams[k % self.inflight])

    def _issue(self, k, count):
        buf = self.bufs[k % self.nbuf]
        with self._stream(k):
            self.render_bands(buf, self.band_rows, self.rank, self.world, k % self.inflight, count)
            if not self.collective:
                return None
            glist = None
            g = self.gathered[k % self.nbuf] if self.rank == 0 else None
            n = count * self.nbytes  # this launch's frames, rank-major: rank i's at i * n
            if self.stage_host:
                host = buf[:n].cpu()  # waits for this launch's render on the stream
                if self.rank == 0:
                    glist = [torch.empty_like(host) for _ in range(self.world)]
                dist.gather(host, gather_list=glist, dst=0, group=self.group)
                if self.rank == 0:
                    g[:self.world * n].copy_(torch.cat(glist))
                return None
            if self.rank == 0:
                glist = [g[i * n:(i + 1) * n] for i in range(self.world)]
            return dist.gather(buf[:n], gather_list=glist, dst=0, group=self.group, async_op=True)

    def _finish(self, k, work, count):
        if self.collective:
            with self._stream(k):
                if work is not None:
                    work.wait()  # NCCL: the stream waits for the gather (the host does not)
                if self.rank == 0:
                    g, fr = self.gathered[k % self.nbuf], self.frames[k % self.nbuf]
                    fb = self.height * self.width * 4
                    for b in range(count):  # frame b of the launch: rank r's at r*count*nbytes + b*nbytes
                        self.unshuffle(g[b * self.nbytes:], count * self.nbytes, fr[b * fb:(b + 1) * fb],
                                       k % self.inflight)
        self.last = k % self.nbuf
        self.last_count = count
        self.frames_done += count

    def run(self, n, before_frame=None, capture=None):
        """Render, gather and reassemble n frames (asynchronous on the GPU path: callers
        synchronize the device to wait for the last one). Launches take `batch` frames each,
        the last one the remainder. before_frame(k), if given, runs on the host before frame k
        is issued (e.g. to advance animated parameters); for a launch of several frames, before
        each of its frames, before the launch. capture (rank 0; a flat uint8 tensor of one
        frame): the first frame of this run is copied into it, in stream order after its
        render (and reassembly), before its buffers are reused."""
        pending = None
        done = 0
        for k in range(-(-n // self.batch)):
            count = min(self.batch, n - done)
            if before_frame is not None:
                for j in range(count):
                    before_frame(done + j)
            done += count
            if pending is not None and pending[0] % self.nbuf == k % self.nbuf:
                # one buffer set (nbuf 1): the previous launch is reassembled and captured in
                # stream order before this launch overwrites its buffer
                self._finish(*pending)
                self._capture(pending[0], capture)
                pending = None
            work = self._issue(k, count)
            if pending is not None:
                self._finish(*pending)
                self._capture(pending[0], capture)
            pending = (k, work, count)
        if pending is not None:
            self._finish(*pending)
            self._capture(pending[0], capture)

    def _capture(self, k, capture):
        if capture is None or k != 0 or (self.collective and self.rank != 0):
            return
        with self._stream(k):
            capture.copy_(self._frame(k % self.nbuf, 0))

    def _frame(self, buf, b):
        """Rank 0: frame b of the launch that used buffer set `buf`, flat RGBA8."""
        if not self.collective:
            return self.bufs[buf][b * self.nbytes:(b + 1) * self.nbytes]
        fb = self.height * self.width * 4
        return self.frames[buf][b * fb:(b + 1) * fb]

    def output(self):
        """Rank 0: the last frame, flat RGBA8 (the band buffer itself when world == 1)."""
        return self._frame(self.last, self.last_count - 1)
