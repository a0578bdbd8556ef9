/*
 * rt_capi.h — the C-ABI drop-in boundary of the MI355X trace/shade path.
 *
 * The reference renders a frame with one C++ call,
 *     void rt_scene(std::vector<vec3> u, const std::vector<std::unique_ptr<SceneGeometry>>& scene,
 *                   const Camera& cam, std::vector<std::vector<RGB>>& frame_buffer);
 * (/root/reference/main.cpp:124-139), which walks every pixel through
 * recursive_ray_tracing (main.cpp:89-119) -> find_closest_hit (main.cpp:67-84) ->
 * the virtual SceneGeometry::intersect plugin (scene.h:57; Sphere::intersect
 * scene.cpp:40-78, Wall::intersect scene.cpp:4-35).
 *
 * This header is what a host program binds instead: plain C, plain pointers and
 * sizes, no C++ or torch types.  The C++ API mirror (include/rt/scene.h) flattens its
 * SceneGeometry objects into rt_prim records and calls these entry points; a cgo /
 * ctypes / N-API binding binds them directly.
 *
 * Conventions (the reference has no error returns; .at() throws — main.cpp:136):
 *   - every entry point returns int status, RT_OK == 0; rt_strerror() names it;
 *   - no exception crosses the boundary;
 *   - a ctx is used by one host thread at a time; calls on a ctx are serialised;
 *   - the caller owns every buffer passed in; the ctx owns its device copies.
 */
#ifndef RT_CAPI_H
#define RT_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Version 2 adds the multi-GPU frame operator (rt_multi_*) and RT_ERR_COMM; every version-1
 * entry point keeps its signature and meaning (the ABI grows additively). */
#define RT_CAPI_VERSION 2

/* ---- status codes ------------------------------------------------------- */
enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID_ARG = 1,   /* null pointer, bad size, bad enum */
    RT_ERR_NO_DEVICE = 2,     /* no HIP device / device index out of range */
    RT_ERR_HIP = 3,           /* a HIP runtime call failed (rt_last_hip_error) */
    RT_ERR_OUT_OF_MEMORY = 4,
    RT_ERR_NO_SCENE = 5,      /* rt_render* before rt_set_scene */
    RT_ERR_UNSUPPORTED = 6,   /* depth / flag combination this build does not ship */
    RT_ERR_OUT_OF_RANGE = 7,  /* row band outside the image (reference: std::out_of_range) */
    RT_ERR_COMM = 8           /* an RCCL call failed (rt_multi_last_error names it) */
};

/* ---- scene records (reference scene.h:35-84) ---------------------------- */

/* Material — scene.h:35-49.  NOTE the reference constructor's positional order is
 * (color, metallic, ambient, diffuse, specular, specular_exponent) with defaults
 * .5/.1/.9/.4/50 (scene.h:48); the fields here are named, so order is irrelevant. */
typedef struct rt_material {
    double color[3];
    double ambient;
    double metallic;
    double diffuse;
    double specular;
    double specular_exponent;
} rt_material;

enum rt_prim_kind {
    RT_PRIM_SPHERE = 0,   /* Sphere, scene.h:75-84 */
    RT_PRIM_WALL = 1      /* Wall,   scene.h:62-73 */
};

/* One SceneGeometry object, flattened.  Fields hold the OBJECT STATE, i.e. what the
 * reference constructors store: Wall's normal is already normalised (scene.h:73
 * normalises in the initialiser list), position is the wall's corner (scene.cpp:30). */
typedef struct rt_prim {
    int32_t kind;          /* rt_prim_kind */
    int32_t reserved;      /* must be 0 */
    rt_material mat;
    double position[3];    /* Sphere::center | Wall::position */
    double normal[3];      /* Wall::normal (unit); ignored for spheres */
    double radius;         /* Sphere::radius */
    double length;         /* Wall::length */
    double width;          /* Wall::width */
} rt_prim;

/* The per-frame camera inputs of rt_scene (main.cpp:132-134): position plus the
 * Camera::init outputs image_top_left and the returned {pixel_delta_x, pixel_delta_y}
 * (scene.cpp:80-106).  They are passed explicitly (not recomputed from lookat)
 * because the reference never re-calls init() after a camera move (main.cpp:154),
 * so a moved camera keeps a stale image_top_left — a drop-in must reproduce that. */
typedef struct rt_camera {
    double position[3];
    double image_top_left[3];
    double pixel_delta_x[3];   /* u[0] in rt_scene */
    double pixel_delta_y[3];   /* u[1] in rt_scene */
    int32_t width;             /* cam.image_width */
    int32_t height;            /* cam.image_height */
} rt_camera;

/* ---- render options ----------------------------------------------------- */
enum rt_precision {
    RT_PREC_F64 = 0,     /* fp64 everywhere, op-for-op the reference's arithmetic (parity) */
    RT_PREC_F32 = 1,     /* fp32 everywhere (throughput; flips at discontinuities) */
    RT_PREC_MIXED = 2,   /* fp32 conservative cull + fp64 exact on survivors: output == F64 */
    RT_PREC_PATH64 = 3   /* F64's exact ray paths (hits, normals, reflections) + fp32 colour
                            arithmetic: no discontinuity flips, colours within ~1e-6 */
};

/* The reference's only post-step is SDL_MapRGB(format, val.x*255, ...) (main.cpp:345),
 * whose Uint8 parameters take the double by implicit conversion.  For 0 <= v*255 < 256
 * that truncates toward zero; above (local colour can reach color*1.4: diffuse .9 +
 * specular .4 + ambient .1) the conversion is undefined in C++, and the reference's
 * x86-64 build (g++ -O3: cvttsd2si, then the low byte) WRAPS modulo 256 — a highlight of
 * 1.084 displays as 20.  RT_OUT_RGBA8 deliberately deviates there and saturates at 255
 * (the tone-map epilogue); RT_OUT_RGBA8_WRAP reproduces the x86-64 bytes exactly
 * (tests/golden/surface.npz, recorded from that conversion compiled by g++). */
enum rt_out_format {
    RT_OUT_RGB_F32 = 0,  /* H x W x 3 float, row-major, linear unclamped RGB (12 B/px) */
    RT_OUT_RGB_F64 = 1,  /* H x W x 3 double (24 B/px) — exact drop-in for vector<vector<RGB>> */
    RT_OUT_RGBA8 = 2,    /* H x W x 4 uint8 (R,G,B,255): trunc(clamp(v,0,1)*255).  Equals
                            main.cpp:345 for in-range pixels; saturates (a deliberate
                            deviation) where the reference's conversion wraps */
    RT_OUT_RGBA8_WRAP = 3 /* H x W x 4 uint8 (R,G,B,255): (uint8)(int32)trunc(v*255), i.e.
                            main.cpp:345's bytes on x86-64 for every value, out-of-range
                            (wraps mod 256) and NaN (0) included */
};

enum rt_flags {
    RT_FLAG_SUN = 1u << 0   /* build-defined sun term (SUN_COLOR/SUN_DIRECTION, main.cpp:18-19,
                               defined but unused by the reference); off = reference parity */
};

typedef struct rt_stats {
    double ms;             /* device time of the render (hipEvent), milliseconds */
    uint64_t segments;     /* closest-hit queries issued (only when counting was asked) */
} rt_stats;

typedef struct rt_ctx rt_ctx;

/* ---- lifecycle ---------------------------------------------------------- */
int rt_ctx_create(int device, rt_ctx** out);
int rt_ctx_destroy(rt_ctx* ctx);
const char* rt_strerror(int status);
const char* rt_last_hip_error(const rt_ctx* ctx);
int rt_capi_version(void);

/* ---- scene -------------------------------------------------------------- */
/* Copies n primitives (in scene order: index j is the reference's scene.at(j)) to the
 * device.  Replaces any previous scene.  n == 0 is a valid (empty) scene.  Waits first
 * for every render this ctx has enqueued, on its own stream and on caller streams
 * (rt_render_device), so frames in flight finish on the old scene. */
int rt_set_scene(rt_ctx* ctx, const rt_prim* prims, int32_t n);

/* ---- tuning ------------------------------------------------------------- */
enum rt_option {
    RT_OPT_WAVE_CULL_MIN_SPHERES = 1, /* scenes with at least this many spheres use the
                                         wave-cooperative cull (default 24; 0 = always,
                                         INT32_MAX = never).  Output is identical. */
    RT_OPT_STATS_DEVICE_PTR = 2,      /* diagnostics: device address of 3 uint64 counters
                                         that renders add to ([0] wave culls, [1] spheres
                                         kept, [2] spheres considered); 0 = off */
    RT_OPT_EYE_TABLES = 3,            /* 1 (default): primary rays use per-frame tables of
                                         their camera-origin terms (small scenes); 0 = off.
                                         Output is identical. */
    RT_OPT_TILE_BINS = 4,             /* 1 (default): per-frame pixel boxes of every
                                         primitive let each 8x8 tile test only what its
                                         primary rays can hit (scenes of <= 64
                                         primitives); 0 = off.
                                         Output is identical. */
    RT_OPT_ROW_ORDER = 5,             /* 1 (default): tile rows are dispatched centre-out
                                         from the estimated heaviest row (scheduling only);
                                         0 = top to bottom.  Output is identical. */
    RT_OPT_MIRROR_BINS = 6,           /* 1 (default): bounces that follow the same wall
                                         chain across a wave use the boxes of the mirrored
                                         camera (needs RT_OPT_TILE_BINS); 0 = off.  Output
                                         is identical. */
    RT_OPT_BOX_CACHE = 7,             /* 1 (default): a render whose scene, camera, band and
                                         options equal the previous render's reuses its
                                         per-frame pixel boxes (host work only); 0 = always
                                         recompute.  Output is identical. */
    RT_OPT_ROW_FEEDBACK = 8,          /* N > 0 (default 32): every render records each
                                         tile's cost; every N frames (and at once for a new
                                         band or scene) a snapshot is copied back behind the
                                         kernel, and later renders of the same band dispatch
                                         tile rows heaviest-first by it (scheduling only);
                                         0 = off.  Setting it (any value) drops the order
                                         and any snapshot still in flight.  Output is
                                         identical. */
    RT_OPT_PIXEL_PAIRS = 9,           /* 1: RT_PREC_PATH64 renders without the wave cull
                                         trace two pixels per lane (16x8 pixels per
                                         wave); 0 (default) = one.  Output is identical. */
    RT_OPT_ROW_FEEDBACK_WARM = 10,    /* K >= 0 (default 0): after a new band or scene,
                                         RT_OPT_ROW_FEEDBACK takes K more snapshots back to
                                         back (each once the previous one has landed)
                                         before its interval applies.  Output is
                                         identical. */
    RT_OPT_WALL_ORDER = 11,           /* 1: the primary scan visits the walls nearest to
                                         the camera first (per frame), so a wall behind the
                                         best hit skips its bounds test; 0 (default) = scene
                                         order (measured: c2 +1% with the order).  Output is
                                         identical (wall ties compare scene indices). */
    RT_OPT_ROW_FEEDBACK_EMA = 14,     /* W in [0, 95] (default 0): the measured row order
                                         ranks tile rows by their cost smoothed over the
                                         band's snapshots, acc = W% acc + (100-W)% new;
                                         0 = the latest snapshot alone.  Output is
                                         identical. */
    RT_OPT_ROW_FEEDBACK_ISOLATE = 15, /* 1: a frame whose tile costs RT_OPT_ROW_FEEDBACK
                                         samples runs alone on the GPU (its stream waits for
                                         this ctx's frames on other streams, and their next
                                         frames wait for it), so the costs are not those of
                                         overlapping frames; 0 (default) = it overlaps like
                                         any frame (measured: the lost overlap costs more
                                         than cleaner costs gain).  Output is identical. */
    RT_OPT_HOST_PIPELINE = 16,       /* 1 (default): rt_render_device_frames computes the
                                         next frames' kernel arguments (pixel boxes, mirror
                                         chains, eye tables) on a helper thread while the
                                         calling thread launches the current frame; 0 = one
                                         thread does both in turn.  The same launches in the
                                         same order: output is identical. */
    RT_OPT_FRAME_BATCH = 21,         /* B in [1, RT_MULTI_BATCH_MAX] (default 1): in
                                         rt_render_device_frames with the host pipeline,
                                         up to B consecutive frames on the same stream that
                                         write distinct buffers go to the GPU as ONE launch
                                         (frame = blockIdx.z; each frame's kernel arguments
                                         in a device table copied in front of the launch),
                                         so the host pays one launch per group instead of
                                         one per frame.  Frames sampled by
                                         RT_OPT_ROW_FEEDBACK, a change of the row order's
                                         grid, wave-cull scenes and RT_OPT_PIXEL_PAIRS launch
                                         one frame at a time.  On rt_multi_set_option: also
                                         a rank renders each RT_OPT_MULTI_BATCH batch's band
                                         frames (and the root its rows) in blocks of B
                                         consecutive frames per stream, over ceil(batch / B)
                                         streams, so each block is one launch.  Output is
                                         identical. */
    RT_OPT_MULTI_FRAMES = 17,        /* rt_multi_set_option only: F in [1, RT_MULTI_SLOTS]
                                         (default 2) band slots per rank — frames of a rank in
                                         flight on F render streams, so a small band's longest
                                         waves (a 1/8 band of config 4: tiles bouncing between
                                         facing walls) overlap F - 1 other frames.  Every
                                         handle of one exchange must use the same F.  The
                                         gathered frames are identical. */
    RT_OPT_MULTI_FAULT = 18,         /* rt_multi_set_option only, a test hook: 1 = the next
                                         frame (or batch) of this handle fails right after
                                         its part of the exchange was queued — the root's
                                         receives, a sender's send (the failure path of a
                                         real exchange on a one-GPU machine). */
    RT_OPT_MULTI_BATCH = 19,         /* rt_multi_set_option only: B in [1,
                                         RT_MULTI_BATCH_MAX] (default 1) frames per gather in
                                         rt_multi_render_device_frames, one process per rank
                                         (nlocal == 1) with contiguous or weighted bands: each
                                         rank renders B frames' bands back to back and sends
                                         them in ONE ncclSend; the root receives every rank's
                                         B bands in one group and scatters them into the B
                                         frames with one kernel.  The per-frame host work of
                                         the exchange (events, RCCL calls: ~20 us per frame,
                                         more than a 1/8 band's kernel) is paid once per B
                                         frames; a frame's rows reach the root when its batch
                                         completes, and a non-root rank's caller stream
                                         follows its batch's send.  A call batches when
                                         B > 1, nframes >= 2 and every camera has the same
                                         size (so every rank decides alike; every handle of
                                         one exchange must use the same B); the root then
                                         needs a DISTINCT frame buffer for each frame of a
                                         batch (min(B, nframes) of them: frames of one batch
                                         sharing a buffer could never be whole in it) and at
                                         most RT_MULTI_SLOTS distinct caller streams, else
                                         the call is refused before anything is enqueued
                                         (RT_ERR_UNSUPPORTED; with ranks in other processes
                                         the exchange is then broken, as the peers' sends of
                                         that call have no receives).  A buffer of an earlier
                                         batch is rendered into again only after that
                                         batch's gather into it completed, so every frame is
                                         whole in its buffer from its batch's end until the
                                         next frame written there (2 B buffers keep
                                         consecutive batches overlapped).  The frames are
                                         identical. */
    RT_OPT_MULTI_TIMEOUT_MS = 20,    /* rt_multi_set_option only: T >= 0 (default 120000)
                                         ms that rt_multi_sync waits for this process's
                                         streams; it polls them (and RCCL's asynchronous
                                         error) and, when T passes or RCCL reports an error,
                                         breaks the exchange, aborts the communicators
                                         (ncclCommAbort) and returns RT_ERR_COMM instead of
                                         blocking forever on a peer that failed.  0 = no
                                         deadline. */
    RT_OPT_MULTI_LAYOUT = 13,        /* rt_multi_set_option only: 0 (default) = contiguous
                                         row bands (rt_band_rows); 1 = interleaved tile rows
                                         (rt_interleaved_rows): balanced when the frame's cost
                                         is concentrated in some rows (config 5); 2 =
                                         contiguous bands cut at tile rows so that each
                                         carries an equal share of the per-tile-row weights
                                         given to rt_multi_set_row_weights
                                         (rt_weighted_band_rows; equal bands while no weights
                                         cover the frame's tile rows).  The gathered frame is
                                         identical. */
    RT_OPT_CLUSTER_COS = 12           /* C in [-2000, 2000] (default 400): in scenes that use
                                         the wave cull, a wave (any precision) whose live
                                         rays' cone has cos(half-angle) < C/1000 tests each
                                         lane's own ray against sphere clusters (boxes of
                                         <= 8 spheres) and runs the exact test on its own
                                         clusters only; -2000 = never (measured: c5 PATH64
                                         -36%, F64 -44%, c3 -4..15% at 300-500).  Output is
                                         identical. */
};
int rt_set_option(rt_ctx* ctx, int32_t option, int64_t value);

/* Explicit dispatch order of the tile rows (8 pixel rows each): perm is a permutation of
 * 0..n-1, used by every render whose band has exactly n tile rows, ahead of
 * RT_OPT_ROW_FEEDBACK; n = 0 clears it.  Scheduling only: output is identical.
 * RT_ERR_INVALID_ARG if perm is not a permutation or n > 2048. */
int rt_set_row_order(rt_ctx* ctx, const int16_t* perm, int32_t n);

/* ---- frame operators (replace rt_scene, main.cpp:124-139) --------------- */
/* Render rows [row0, row0+nrows) of the frame into caller-owned HOST memory `out`
 * (nrows*width pixels of `out_format`), synchronously.  depth = remaining_iterations
 * of recursive_ray_tracing (rt_scene passes the default 10, main.cpp:89/136).
 * stats may be NULL; stats->segments is filled only when count_segments != 0. */
int rt_render(rt_ctx* ctx, const rt_camera* cam, int32_t row0, int32_t nrows, int32_t depth,
              int32_t precision, uint32_t flags, int32_t out_format, void* out,
              int32_t count_segments, rt_stats* stats);

/* Same, but `d_out` is DEVICE memory and the launch is enqueued on `stream`
 * (a hipStream_t; NULL = the ctx's stream) without synchronising: the hot path as a
 * bench or a multi-GPU tiler drives it.  If d_segments != NULL it must point to one
 * device uint64 that receives += the segment count.  The launch signals a per-stream
 * event of the ctx that rt_set_scene / rt_ctx_destroy wait on (up to 16 streams are
 * tracked; a 17th retires the oldest by waiting on it).  Every entry point runs on the
 * ctx's device and leaves the caller's current device unchanged. */
int rt_render_device(rt_ctx* ctx, const rt_camera* cam, int32_t row0, int32_t nrows,
                     int32_t depth, int32_t precision, uint32_t flags, int32_t out_format,
                     void* d_out, uint64_t* d_segments, void* stream);

/* A batch of frames of the frame loop (main.cpp:250-375 renders one frame per iteration),
 * enqueued by one call: frame f (0 <= f < nframes) renders cams[f % ncams] into
 * d_outs[f % nouts] on streams[f % nstreams] (NULL entries = the ctx's stream), exactly
 * as nframes rt_render_device calls in that order would — each frame's own host work
 * (pixel boxes, row order) and launch — without the caller's per-call overhead.  No
 * synchronisation; stops at the first failing frame and returns its status. */
int rt_render_device_frames(rt_ctx* ctx, const rt_camera* cams, int32_t ncams, int32_t row0,
                            int32_t nrows, int32_t depth, int32_t precision, uint32_t flags,
                            int32_t out_format, void* const* d_outs, int32_t nouts,
                            void* const* streams, int32_t nstreams, int32_t nframes);

/* ---- multi-GPU frame operator (BASELINE config 4) ----------------------- */
/* ONE frame split into contiguous row bands (rt_band_rows) over nranks ranks, one GPU each,
 * every band rendered by that rank's own rt_ctx, then gathered into the frame buffer of
 * rank 0 (the root) — the reference renders the frame on one CPU thread (main.cpp:124-139,
 * called at main.cpp:329); pixels are independent, so the gathered frame is bitwise the
 * one-GPU frame.  Two process models, one object:
 *   - one process drives every GPU: nlocal == nranks, first_rank 0, unique_id NULL
 *     (the communicator is made as ncclCommInitAll would; one host worker thread per extra
 *     device does that rank's per-frame host work and launches in parallel);
 *   - one process per GPU (torchrun-style): nlocal == 1, first_rank = this process's rank,
 *     unique_id = the RT_MULTI_ID_BYTES bytes rt_multi_unique_id returned on ONE process
 *     and shared with the others (ncclCommInitRank; blocks until every rank has joined).
 * Transports: RT_TRANSPORT_RCCL gathers with ncclSend/ncclRecv (rccl.h) over xGMI —
 * bands may differ in height by one row, so no padding; RT_TRANSPORT_COPY (one process
 * only) copies each band into the root's frame with hipMemcpyPeerAsync and also accepts
 * the same device more than once (several ranks on one GPU: the orchestration without
 * RCCL, e.g. on a one-GPU machine); RT_TRANSPORT_RCCL_LOOPBACK is RT_TRANSPORT_RCCL with
 * the root's own band also sent through RCCL (a self ncclSend/ncclRecv pair in the same
 * group as the other bands' receives) and a communicator even at one rank — so every RCCL
 * call of the gather (ncclCommInitRank, the group, send/recv, ncclCommGetAsyncError)
 * executes on a one-GPU machine; it costs one extra copy of the root's band.
 * Frames in flight: each non-root rank renders into one of RT_OPT_MULTI_FRAMES (<=
 * RT_MULTI_SLOTS) band buffers, each with its own render stream, while earlier frames' bands
 * are still being rendered or sent on its comm stream;
 * a band buffer is reused only after its send has completed (device-side event waits; the
 * host never blocks in rt_multi_render_device*).
 * Failures: argument checks every rank makes alike return their status and leave the
 * rt_multi usable.  A frame that fails after them leaves the exchange out of step when any
 * rank may have queued its part (a receive or a send): always with ranks in other processes
 * (they queue theirs whatever this process did), and with every rank in this process once
 * a local rank queued its part.  The rt_multi is then broken — every later frame returns
 * RT_ERR_COMM, rt_multi_sync aborts the communicator (ncclCommAbort) instead of waiting on
 * receives that cannot complete, and rt_multi_destroy aborts instead of destroying.  With
 * one process per GPU over RCCL the other processes are not told: their rt_multi_sync
 * polls their streams and RCCL's asynchronous error and gives up at its deadline
 * (RT_OPT_MULTI_TIMEOUT_MS: broken, communicator aborted, RT_ERR_COMM).  The mailbox
 * transports (THREADS, IPC) tell every peer at once: their waits return RT_ERR_COMM. */
#define RT_MULTI_ID_BYTES 128
#define RT_MULTI_SLOTS 4   /* band slots per rank (RT_OPT_MULTI_FRAMES uses 1..4, default 2) */
#define RT_MULTI_BATCH_MAX 16  /* frames per gather (RT_OPT_MULTI_BATCH) */
enum rt_transport {
    RT_TRANSPORT_RCCL = 0,
    RT_TRANSPORT_COPY = 1,
    RT_TRANSPORT_RCCL_LOOPBACK = 2,
    /* Rehearsal of the one-process-per-GPU model inside ONE process: every rank is its own
     * rt_multi handle (nlocal = 1, first_rank = its rank, the same unique_id, which keys an
     * in-process mailbox), each driven from its own thread as a separate process would drive
     * it, and each ncclSend/ncclRecv pair is a peer copy matched through the mailbox (the
     * root posts where the part lands and after which event; the sender's comm stream waits
     * for it, copies, and posts its completion event, which the root's comm stream waits
     * on).  Handles may share a device.  The host calls of a frame block until the peer's
     * matching post (RCCL's never block); a handle's failure or destroy ends the exchange
     * for all of them (RT_ERR_COMM, no hang). */
    RT_TRANSPORT_THREADS = 3,
    /* Rehearsal of the one-process-per-GPU model ACROSS processes, one per rank (nlocal = 1,
     * first_rank = its rank, the same unique_id — any RT_MULTI_ID_BYTES bytes the processes
     * share, e.g. random ones — naming a POSIX shared-memory mailbox; at most 64 ranks).
     * The THREADS protocol between processes: the root's staging buffers and every rank's
     * exchange events are shared once with hipIpcGetMemHandle / hipIpcGetEventHandle; a
     * sender's comm stream waits on the root's "ready" event, copies its part into the
     * root's staging buffer and records its "sent" event, on which the root's comm stream
     * waits before copying the part into the frame rows.  Processes may share a device (one
     * GPU).  rt_multi_create blocks until every rank has joined; the segment's name is
     * removed once all have.  A rank's failure ends the exchange for all of them
     * (RT_ERR_COMM); a peer process that exits is detected. */
    RT_TRANSPORT_IPC = 4
};
typedef struct rt_multi rt_multi;

/* A fresh communicator id (ncclGetUniqueId) for the one-process-per-GPU model. */
int rt_multi_unique_id(uint8_t id[RT_MULTI_ID_BYTES]);

/* devices[nlocal]: the HIP device of each local rank (global ranks first_rank ..
 * first_rank + nlocal - 1 of nranks).  RT_ERR_NO_DEVICE for a device index out of range,
 * RT_ERR_UNSUPPORTED for RT_TRANSPORT_RCCL with a device listed twice or
 * RT_TRANSPORT_COPY across processes, RT_ERR_COMM if RCCL fails. */
int rt_multi_create(const int32_t* devices, int32_t nlocal, int32_t nranks, int32_t first_rank,
                    const uint8_t* unique_id, int32_t transport, rt_multi** out);
int rt_multi_destroy(rt_multi* m);
const char* rt_multi_last_error(const rt_multi* m);

/* rt_set_scene / rt_set_option on every local rank's ctx (each rank keeps its own per-band
 * state: tile boxes, measured row order). */
int rt_multi_set_scene(rt_multi* m, const rt_prim* prims, int32_t n);
int rt_multi_set_option(rt_multi* m, int32_t option, int64_t value);

/* Enqueue one frame.  d_frame: on the process holding the root, DEVICE memory on the root's
 * device of height x width pixels of out_format (the root's band is rendered into it in
 * place, the other bands are received into their rows); NULL on other processes.  stream
 * (a hipStream_t on the root's device; NULL = the root ctx's stream): the frame's work
 * starts after the work already on it, and work enqueued on it later sees the complete
 * frame.  On a process without the root, a non-NULL stream (on that rank's device) waits for
 * the rank's band to have been sent.  No host synchronisation. */
int rt_multi_render_device(rt_multi* m, const rt_camera* cam, int32_t depth, int32_t precision,
                           uint32_t flags, int32_t out_format, void* d_frame, void* stream);

/* nframes frames as rt_multi_render_device calls in order would enqueue them: frame f
 * renders cams[f % ncams] into d_frames[f % nbufs] on streams[f % nstreams]. */
int rt_multi_render_device_frames(rt_multi* m, const rt_camera* cams, int32_t ncams,
                                  int32_t depth, int32_t precision, uint32_t flags,
                                  int32_t out_format, void* const* d_frames, int32_t nbufs,
                                  void* const* streams, int32_t nstreams, int32_t nframes);

/* Synchronous: the gathered frame in caller-owned HOST memory `out` (height x width pixels
 * of out_format) on the process holding the root (out may be NULL elsewhere).
 * stats->ms = device time from the start of the frame's work to the complete frame on the
 * root (render + gather); stats->segments is not counted (0). */
int rt_multi_render(rt_multi* m, const rt_camera* cam, int32_t depth, int32_t precision,
                    uint32_t flags, int32_t out_format, void* out, rt_stats* stats);

/* Waits for every frame this process enqueued; RT_ERR_COMM if RCCL reported an
 * asynchronous error. */
int rt_multi_sync(rt_multi* m);

/* Per-tile-row weights (n = tile rows of the frames to come, rt_tile_rows() pixel rows each)
 * for RT_OPT_MULTI_LAYOUT = 2, e.g. rt_tile_row_costs of one GPU's render of the frame.
 * Every rank must be given the same weights (one process per GPU: broadcast them).  n = 0
 * clears them.  Frames in flight keep the bands they started with. */
int rt_multi_set_row_weights(rt_multi* m, const float* weights, int32_t n);

/* Contiguous band of `rank` whose boundaries fall on tile rows: boundary r (0 < r < nranks)
 * is the tile row t whose prefix sum of weights[0..t) is nearest r/nranks of the total (ties
 * to the lower t; boundaries never decrease).  weights must hold one entry >= 0 per tile row
 * of `height` (n == ceil(height / rt_tile_rows())); otherwise RT_ERR_INVALID_ARG. */
int rt_weighted_band_rows(int32_t height, int32_t nranks, int32_t rank, const float* weights,
                          int32_t n, int32_t* row0, int32_t* nrows);

/* Measured cost of every tile row of the frame (synchronous): one render of the whole frame
 * by the stamped kernels, in which every wave records its shader cycles; costs[t] = the sum
 * over tile row t's waves in units of 32 cycles.  n must be ceil(height / rt_tile_rows()). */
int rt_tile_row_costs(rt_ctx* ctx, const rt_camera* cam, int32_t depth, int32_t precision,
                      uint32_t flags, float* costs, int32_t n);

/* Interleaved parts: the frame's tile rows (rt_tile_rows() = 8 pixel rows each; the last may be shorter)
 * dealt round-robin to nparts parts — part p owns tile rows p, p + nparts, p + 2 nparts, ...
 * — so every part gets a share of the frame's heavy and light rows (rt_multi's balanced
 * layout, RT_OPT_MULTI_LAYOUT).  *nrows = the part's pixel rows. */
int rt_interleaved_rows(int32_t height, int32_t nparts, int32_t part, int32_t* nrows);

/* rt_render_device for interleaved part `part` of `nparts`: out_frame_rows == 0 stores the
 * part's rows back to back in frame order (rt_interleaved_rows x width pixels in d_out);
 * != 0 stores every row at its frame row (d_out is the whole frame; the other parts' rows
 * are not touched).  nparts == 1 is the whole frame. */
int rt_render_device_interleaved(rt_ctx* ctx, const rt_camera* cam, int32_t nparts, int32_t part,
                                 int32_t depth, int32_t precision, uint32_t flags,
                                 int32_t out_format, void* d_out, int32_t out_frame_rows,
                                 uint64_t* d_segments, void* stream);

/* ---- host helpers (restatements the host side of rt_scene needs) -------- */
/* Camera::init (scene.cpp:80-106) in fp64: fills cam from the Camera fields.
 * height = (int)(image_width / aspect_ratio) exactly as scene.cpp:82. */
int rt_camera_init(const double position[3], const double lookat[3], const double vup[3],
                   double vfov, double aspect_ratio, double image_width, rt_camera* cam);

/* Bytes per pixel of an output format (0 for an unknown format). */
int32_t rt_out_bytes_per_pixel(int32_t out_format);

/* Row band owned by `rank` of `nranks` when the frame is split into contiguous
 * blocks for multi-GPU tiling: [*row0, *row0 + *nrows). */
int rt_band_rows(int32_t height, int32_t nranks, int32_t rank, int32_t* row0, int32_t* nrows);

/* Diagnostics, host only (no device): the per-frame pixel boxes of the tile bins for a
 * scene and camera, as the linear-scan kernels would receive them (<= 64 primitives, else
 * *nbox = 0).  out receives 4 int16 per box {x0, x1, i0, i1} (inclusive pixel column and
 * frame row ranges; x0 > x1 = never hit): the *nbox primary boxes in material-slot order
 * (spheres in scene order, then walls in scene order, z-normal walls that can never be hit
 * dropped), then for each mirror level L = 1..*mir_depth the nW^L wall sequences (base-nW
 * number w1..wL) of *nbox boxes each.  RT_ERR_INVALID_ARG when cap (boxes) is too small
 * (*nbox and *mir_depth are still set). */
int rt_frame_boxes(const rt_prim* prims, int32_t n, const rt_camera* cam, int32_t row0,
                   int32_t nrows, int16_t* out, int32_t cap, int32_t* nbox, int32_t* mir_depth);

/* Largest depth the kernels are compiled for (depth 0..rt_max_depth()). */
int32_t rt_max_depth(void);

/* Pixel rows per tile row of the kernels (the unit rt_interleaved_rows deals, 8). */
int32_t rt_tile_rows(void);

/* ---- diagnostics -------------------------------------------------------- */
/* Device self-test of the fp64 helpers the exact path relies on, over n seeded random
 * operands: test 0 = division with a shared refined reciprocal vs IEEE `/` (bitwise),
 * test 1 = integer-exponent pow by squaring vs pow() (within 128 ulp),
 * test 2 = the range-restricted sqrt sequence vs sqrt() (bitwise).
 * *mismatches receives the number of failures (0 expected). */
int rt_selftest(rt_ctx* ctx, int32_t test, uint64_t n, uint64_t seed, uint64_t* mismatches);

#ifdef __cplusplus
}
#endif
#endif /* RT_CAPI_H */
