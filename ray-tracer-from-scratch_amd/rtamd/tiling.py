"""Multi-GPU row tiling of ONE frame (BASELINE config 4): one process per GPU, each rank
renders a contiguous band of rows (rt_band_rows) into device memory through the C-ABI,
then the bands are gathered to one rank over RCCL (torch.distributed backend "nccl").

The reference has no multi-GPU path (no collectives); this is the build's one
exchange step.  Pixels are independent, so the assembled frame is bitwise the 1-GPU frame.

* `gather_frame` — one frame, synchronous; the band renderer is a callable, so the same
  code runs with the HIP path on GPUs and with any CPU renderer over gloo in tests.
* `TiledFrames` — frames back to back with N-deep buffering: the gather of frame k runs
  asynchronously (on the collective's own stream) while frame k+1 renders; when the
  height divides evenly the bands land directly in row slices of the destination frame
  (no assembly copy).
"""
from __future__ import annotations

from typing import Callable, Optional

from . import capi


def band_of(height: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous row band [row0, row0 + nrows) of `rank` (rt_band_rows)."""
    return capi.band_rows(height, world, rank)


def gather_frame(render_band: Callable[[int, int, "object"], None], height: int, width: int,
                 channels: int, dtype, device, group=None, dst: int = 0):
    """Render this rank's band with render_band(row0, nrows, out_tensor) and gather every
    band to `dst`.  Returns the (height, width, channels) frame on dst, None elsewhere.

    Bands differ by at most one row; each is padded to the largest so one fixed-size
    gather moves them (RCCL/gloo gather needs equal sizes)."""
    t = TiledFrames(render_band, height, width, channels, dtype, device, group, dst, depth=1)
    t.wait(t.submit())
    return t.frame(0)


class TiledFrames:
    """Row-tiled frames with `depth`-deep buffering (see module doc).

    submit() renders this rank's band of the next frame into buffer slot k % depth and
    starts its gather asynchronously; wait(handle) completes it (and, for uneven bands,
    assembles the frame on dst); frame(slot) is the assembled frame on dst."""

    def __init__(self, render_band, height, width, channels, dtype, device, group=None,
                 dst=0, depth=2):
        import torch
        import torch.distributed as dist
        self.dist = dist
        self.render_band = render_band
        self.h, self.w, self.c = height, width, channels
        self.group, self.dst, self.depth = group, dst, depth
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.row0, self.nrows = band_of(height, self.world, self.rank)
        self.maxrows = -(-height // self.world) if height else 0
        self.even = height % self.world == 0
        is_dst = self.rank == dst
        self.frames = [torch.empty((height, width, channels), dtype=dtype, device=device)
                       if is_dst else None for _ in range(depth)]
        if self.even:
            # bands are row slices of the frame: contiguous, gathered in place on dst
            if is_dst:
                self.bands = [f[self.row0:self.row0 + self.nrows] for f in self.frames]
                self.lists = [[f[r * self.maxrows:(r + 1) * self.maxrows]
                               for r in range(self.world)] for f in self.frames]
            else:
                self.bands = [torch.empty((self.maxrows, width, channels), dtype=dtype,
                                          device=device) for _ in range(depth)]
                self.lists = [None] * depth
        else:
            self.bands = [torch.zeros((self.maxrows, width, channels), dtype=dtype,
                                      device=device) for _ in range(depth)]
            self.lists = [[torch.empty_like(self.bands[0]) for _ in range(self.world)]
                          if is_dst else None for _ in range(depth)]
        self.k = 0
        self.pending = [None] * depth

    def submit(self):
        slot = self.k % self.depth
        if self.pending[slot] is not None:      # slot reused: its previous gather must end
            self.wait(self.pending[slot])
        if self.nrows:
            self.render_band(self.row0, self.nrows, self.bands[slot])
        work = self.dist.gather(self.bands[slot], self.lists[slot], dst=self.dst,
                                group=self.group, async_op=True)
        handle = (slot, work)
        self.pending[slot] = handle
        self.k += 1
        return handle

    def wait(self, handle):
        slot, work = handle
        if self.pending[slot] is not handle:
            return
        work.wait()
        self.pending[slot] = None
        if not self.even and self.rank == self.dst:
            f = self.frames[slot]
            for r, g in enumerate(self.lists[slot]):
                a, n = band_of(self.h, self.world, r)
                if n:
                    f[a:a + n].copy_(g[:n])

    def drain(self):
        for h in list(self.pending):
            if h is not None:
                self.wait(h)

    def frame(self, slot: int):
        return self.frames[slot]


def render_tiled(renderer: "capi.Renderer", cam, depth: int, precision: int = capi.RT_PREC_PATH64,
                 flags: int = 0, out_format: int = capi.RT_OUT_RGB_F32, group=None, dst: int = 0,
                 stream: Optional[object] = None):
    """Row-tiled render of one frame on the GPUs of `group` (HIP path), gathered to dst."""
    import torch
    dt_np, shape = capi.out_dtype_shape(out_format, 1, cam.width)
    tdtype = {"float32": torch.float32, "float64": torch.float64, "uint8": torch.uint8}[
        dt_np.__name__]
    dev = torch.device("cuda", torch.cuda.current_device())
    # never the legacy default stream (handle 0): the C-ABI maps a NULL stream to the ctx's
    # own non-blocking stream, which nothing on the torch side would be ordered with
    st = stream if stream is not None and stream.cuda_stream != 0 else torch.cuda.Stream(dev)

    def band(row0, nrows, out):
        cur = torch.cuda.current_stream(dev)
        if st != cur:
            st.wait_stream(cur)  # the band buffer was produced (zeroed) on the current stream
        renderer.render_device(cam, depth, out.data_ptr(), precision, flags, out_format,
                               row0=row0, nrows=nrows, stream=st.cuda_stream)
        if st != cur:
            # ProcessGroupNCCL orders the gather after the CURRENT stream only: make it wait
            # for the band's kernel on the render stream
            cur.wait_stream(st)

    return gather_frame(band, cam.height, cam.width, shape[-1], tdtype, dev, group, dst)
