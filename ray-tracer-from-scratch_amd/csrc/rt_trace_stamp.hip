/* rt_trace_stamp.hip — the trace kernels of rt_trace.hip built a second time (namespace
 * rt::kst) with each wave recording its cost (shader cycles) into KParams::tile_cost: the
 * frames whose costs the host samples for the tile-row dispatch order (rt_capi.cpp row
 * feedback) launch these, every other frame the plain kernels. */
#define RT_STAMP 1
#include "rt_trace.hip"
