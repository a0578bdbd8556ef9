"""Multi-GPU row tiling of ONE frame (BASELINE config 4): one process per GPU, each rank
renders a contiguous band of rows (rt_band_rows) into device memory through the C-ABI,
then the bands are gathered to one rank over RCCL (torch.distributed backend "nccl").

The reference has no multi-GPU path (no collectives); this is the build's one
exchange step.  Pixels are independent, so the assembled frame is bitwise the 1-GPU frame.

The gather logic is independent of who renders a band: `gather_frame` takes a band
renderer callable, so the same code runs with the HIP path on GPUs (`render_tiled`) and
with any CPU renderer over gloo in the multi-process tests.
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
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    row0, nrows = band_of(height, world, rank)
    maxrows = -(-height // world) if height else 0
    band = torch.zeros((maxrows, width, channels), dtype=dtype, device=device)
    if nrows:
        render_band(row0, nrows, band)
    gather_list = ([torch.empty_like(band) for _ in range(world)] if rank == dst else None)
    dist.gather(band, gather_list, dst=dst, group=group)
    if rank != dst:
        return None
    frame = torch.empty((height, width, channels), dtype=dtype, device=device)
    for r, g in enumerate(gather_list):
        a, n = band_of(height, world, r)
        if n:
            frame[a:a + n].copy_(g[:n])
    return frame


def render_tiled(renderer: "capi.Renderer", cam, depth: int, precision: int = capi.RT_PREC_PATH64,
                 flags: int = 0, out_format: int = capi.RT_OUT_RGB_F32, group=None, dst: int = 0,
                 stream: Optional[object] = None):
    """Row-tiled render of one frame on the GPUs of `group` (HIP path), gathered to dst."""
    import torch

    dt_np, shape = capi.out_dtype_shape(out_format, 1, cam.width)
    tdtype = {"float32": torch.float32, "float64": torch.float64, "uint8": torch.uint8}[
        dt_np.__name__]
    dev = torch.device("cuda", torch.cuda.current_device())
    st = stream or torch.cuda.current_stream(dev)

    def band(row0, nrows, out):
        renderer.render_device(cam, depth, out.data_ptr(), precision, flags, out_format,
                               row0=row0, nrows=nrows, stream=st.cuda_stream)

    return gather_frame(band, cam.height, cam.width, shape[-1], tdtype, dev, group, dst)
