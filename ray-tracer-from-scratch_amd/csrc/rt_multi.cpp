/*
 * rt_multi.cpp — the multi-GPU frame operator of include/rt_capi.h (rt_multi_*):
 * BASELINE config 4, one frame split into contiguous row bands across GPUs and gathered
 * into rank 0's frame buffer.
 *
 * The reference renders every frame on one CPU thread (rt_scene, main.cpp:124-139, called
 * from the event loop at main.cpp:329) and has no multi-device path; this file
 * is the build's one exchange step.  It sits ABOVE the single-GPU C-ABI: every rank is a
 * plain rt_ctx driven through rt_set_scene / rt_set_option / rt_render_device, so a band
 * is rendered by exactly the kernels and host work of a one-GPU render of those rows, and
 * the gathered frame is bitwise the one-GPU frame (pixels are independent).
 *
 * Per frame and rank (stream order does the synchronisation; the host never waits):
 *   root (global rank 0): its band is rendered in place into the caller's frame buffer on
 *     the caller's stream; RCCL: the comm stream waits for the caller's earlier work (the
 *     buffer may still be read), receives every other band into its rows (one
 *     ncclGroupStart/End), and the caller's stream waits for it.
 *   other ranks: slot s's render stream waits until band buffer s has been sent (frame
 *     k - slots, RT_OPT_MULTI_FRAMES), renders the band into it, and the comm stream sends it once the
 *     render is done (RCCL ncclSend, or a peer copy into the root's rows for
 *     RT_TRANSPORT_COPY) — so the render of frame k+1 overlaps the send of frame k, and the
 *     tail of frame k's band kernel (one slot's stream) overlaps frame k+1's (the other's).
 * One process driving several GPUs runs the extra ranks' host work (pixel boxes, row order,
 * launch: rt_render_device) on one worker thread per rank, in parallel with the caller's
 * thread, which does the root's.
 *
 * RT_TRANSPORT_THREADS (rehearsal): the process-per-GPU structure — one rt_multi handle per
 * rank, nlocal = 1, non-root handles without a frame buffer — with the handles living in ONE
 * process, each driven from its own thread, and every ncclSend/ncclRecv pair replaced by a
 * peer copy matched through an in-process mailbox (Hub, keyed by the unique id): the root
 * posts where frame k's part of rank g lands and the event after which it may be written;
 * the sender's comm stream waits for that event, copies, and posts its completion event, on
 * which the root's comm stream waits.  So a one-GPU box runs every branch a process-per-GPU
 * RCCL run takes (the non-root enqueue, the caller-stream wait on the send, the root's
 * interleaved staging and scatter) except the RCCL calls themselves.
 *
 * RT_TRANSPORT_IPC (rehearsal across processes): the same mailbox protocol between real
 * processes, one per rank, on one GPU or several.  The mailbox is a POSIX shared-memory
 * segment named after the unique id (one ring of posts per direction and non-root rank);
 * the root's staging buffers are shared with hipIpcGetMemHandle (once per allocation).  The
 * cross-process stream ordering uses two sequence counters per rank in the same segment,
 * set and awaited ON the streams by host functions (hipLaunchHostFunc): the root's comm
 * stream sets "ready" once the destination may be written; the sender's comm stream waits
 * for it, copies its part into the root's staging buffer through the imported mapping and
 * sets "sent"; the root's comm stream waits for that before copying the part into the frame
 * rows.  (HIP's own IPC events were used first: after ~1,000 frames a wait on an imported
 * event failed with "invalid argument", so the ordering is now this file's own.)  So
 * bench.py's process-per-GPU code (its non-root branches, the broadcasts of the id and the
 * row weights) runs in separate processes on a one-GPU box.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <new>
#include <thread>
#include <vector>

#include "../../include/rt_capi.h"

namespace {

struct Rank;

struct Job {
    const rt_camera* cam = nullptr;
    int32_t depth = 0, precision = 0, out_format = 0;
    uint32_t flags = 0;
    char* d_frame = nullptr;        // root's frame buffer (root rank's job, COPY targets)
    hipStream_t stream = nullptr;   // caller stream (root's device, or this rank's device)
    hipEvent_t ev_in = nullptr;     // recorded on the caller's stream before the frame
    int slot = 0;
};

struct Rank {
    int rank = 0;                   // global rank
    int device = 0;
    rt_ctx* ctx = nullptr;
    ncclComm_t comm = nullptr;
    // one render stream per band slot: consecutive frames' band kernels overlap, so a rank's
    // frame rate is not bounded by its heaviest wave's latency (a c2 band's kernel takes
    // ~20 us for 1/8 of the frame: the tail, tools/band_model.py)
    hipStream_t render_stream[RT_MULTI_SLOTS] = {};
    hipStream_t comm_stream = nullptr;
    void* band[RT_MULTI_SLOTS] = {};
    size_t band_cap = 0;
    hipEvent_t ev_rendered[RT_MULTI_SLOTS] = {};
    hipEvent_t ev_sent[RT_MULTI_SLOTS] = {};
    hipEvent_t ev_done = nullptr;   // root, RCCL / THREADS: every band received
    hipEvent_t ev_ready[RT_MULTI_SLOTS] = {};  // root, THREADS: parts may land
    // root, RCCL, interleaved layout: every rank's part received here, then scattered into
    // its frame rows (one strided copy per part)
    void* staging[RT_MULTI_SLOTS] = {};
    size_t staging_cap = 0;
    // batched gather (RT_OPT_MULTI_BATCH), two batch slots: a sender's bands of the batch's
    // frames back to back (bbuf), the root's received parts (bstage); ev_brend[slot][j]: the
    // batch's bands on render stream j rendered, ev_bsent: its send complete (bbuf free again)
    void* bbuf[2] = {};
    size_t bbuf_cap = 0;
    void* bstage[2] = {};
    size_t bstage_cap = 0;
    hipEvent_t ev_brend[2][RT_MULTI_SLOTS] = {}, ev_bsent[2] = {};
    // root: batch slot b's scatter into its frames is complete (a later batch renders into
    // one of those frame buffers only after it, so every frame is whole in its buffer)
    hipEvent_t ev_bdone[2] = {};
    // rt_multi_sync: recorded on each render stream and the comm stream, then polled
    hipEvent_t ev_drain[RT_MULTI_SLOTS + 1] = {};
    // root, RT_OPT_FRAME_BATCH: its rows of a batch's block of frames rendered (per stream)
    hipEvent_t ev_rows[RT_MULTI_SLOTS] = {};
    // worker thread (local ranks other than the first, one process driving several GPUs)
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<uint64_t> posted{0}, finished{0};
    bool quit = false;
    Job job;
    int status = RT_OK;
};

/* RT_TRANSPORT_THREADS mailbox shared by the handles of one unique id (see the file
 * comment).  Keys are (frame number of the handles, sending rank): every handle counts the
 * frames it renders, and the handles of one exchange render the same sequence. */
struct Post {
    void* dst = nullptr;      // root: where the part lands
    int device = 0;           // root's device
    size_t bytes = 0;
    hipEvent_t ev = nullptr;  // root -> sender: the destination may be written after it;
                              // sender -> root: the copy is complete after it
    const void* owner = nullptr;  // the posting handle (its posts go when it is destroyed)
};
struct Hub {
    std::mutex mu;
    std::condition_variable cv;
    std::map<std::pair<uint64_t, int>, Post> recv, sent;
    int refs = 0;
    bool failed = false;      // a handle failed mid-exchange or was destroyed: waits give up
};
std::mutex g_hubs_mu;
std::map<std::string, std::shared_ptr<Hub>> g_hubs;

/* RT_TRANSPORT_IPC mailbox: one shared-memory segment per unique id, zero-filled by
 * ftruncate and accessed with __atomic builtins only (plain fields, no constructors run in
 * shared memory).  Each non-root rank g has two single-producer rings: `recv` (the root posts
 * where g's part of a frame/batch lands) and `sent` (g posts that its copy was enqueued). */
constexpr int IPC_MAX_RANKS = 64;
constexpr int IPC_RING = 16;
// the exchange events of a rank by index (THREADS posts name one): ev_ready[slot] (root),
// ev_sent[slot], ev_bsent[b]
enum : int { EV_READY = 0, EV_SENT = RT_MULTI_SLOTS, EV_BSENT = 2 * RT_MULTI_SLOTS, IPC_NEV = EV_BSENT + 2 };
struct IpcMsg {
    uint64_t seq;       // n + 1 once message n of the ring is written (release)
    uint64_t frame, bytes, offset;
    uint32_t alloc;     // root -> sender: id of the root's exported staging allocation
    int32_t ev;         // the poster's event (EV_*) to wait on
    hipIpcMemHandle_t mem;  // root -> sender: that allocation's handle
};
struct IpcRing {
    IpcMsg msg[IPC_RING];
    uint64_t taken;     // messages consumed (release)
};
struct IpcPeer {
    uint32_t joined, left;  // set once (release): joined / its imports closed
    int32_t pid, nranks;
    // stream-order counters for this (non-root) rank's posts, set by host functions on the
    // streams: ready = post n's destination may be written (root), sent = post n's copy has
    // landed (sender); value n + 1
    uint64_t ready, sent;
    IpcRing recv, sent_ring;
};
struct IpcShared {
    uint32_t failed;        // a handle failed mid-exchange: every wait gives up
    int32_t failed_rank;
    IpcPeer peer[IPC_MAX_RANKS];
};
struct Ipc {
    IpcShared* sh = nullptr;
    std::string name;
    bool unlinked = false, joined = false;
    struct Exp {
        void* base;
        size_t bytes;
        uint32_t id;
        hipIpcMemHandle_t h;
    };
    std::vector<Exp> exp;                 // root: exported staging allocations (freed at destroy)
    uint32_t next_id = 1;
    std::map<uint32_t, void*> opened;     // sender: the root's allocations mapped here
    std::vector<uint64_t> nrecv, nsent;   // root: posts made / taken per rank
    uint64_t nrecv_taken = 0, nsent_posted = 0;  // sender
};

}  // namespace

struct rt_multi {
    int nranks = 1, nlocal = 1, first_rank = 0, transport = RT_TRANSPORT_RCCL;
    int slots = 2;                  // RT_OPT_MULTI_FRAMES: band slots in use (frames in flight)
    int batch = 1;                  // RT_OPT_MULTI_BATCH: frames per gather
    int frame_batch = 1;            // RT_OPT_FRAME_BATCH (forwarded to every ctx as well)
    uint64_t nbatch = 0;            // batches gathered (batch slot = nbatch % 2)
    bool fault_next = false;        // RT_OPT_MULTI_FAULT (test hook)
    int layout = 0;                 // RT_OPT_MULTI_LAYOUT: 0 contiguous bands, 1 interleaved,
                                    // 2 contiguous bands weighted by `weights`
    std::vector<float> weights;     // rt_multi_set_row_weights: per tile row
    std::vector<Rank*> r;           // local ranks, r[0] = first_rank
    uint64_t frame = 0;
    hipEvent_t ev_in[RT_MULTI_SLOTS] = {};  // root's device (process with root)
    hipStream_t host_stream = nullptr;                       // rt_multi_render (root's device)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    void* d_frame = nullptr;
    size_t d_frame_cap = 0;
    char last_err[320] = {0};
    // a frame failed after some rank may have queued its part of the gather: the
    // communicator is out of step (see rt_capi.h); `aborted` once ncclCommAbort has run
    bool broken = false, aborted = false;
    // set once any local rank has queued its part of this frame's exchange (a receive, a send
    // or a mailbox post): only a failure after that leaves the peers out of step
    std::atomic<bool> queued{false};
    std::shared_ptr<Hub> hub;       // RT_TRANSPORT_THREADS
    std::string hub_key;
    std::unique_ptr<Ipc> ipc;       // RT_TRANSPORT_IPC
    int64_t timeout_ms = 120000;    // RT_OPT_MULTI_TIMEOUT_MS (rt_multi_sync's deadline)
    std::vector<char*> batch_bufs[2];  // root: the frame buffers of batch slot 0 / 1
    bool has_root() const { return first_rank == 0; }
    bool rccl() const { return transport == RT_TRANSPORT_RCCL || transport == RT_TRANSPORT_RCCL_LOOPBACK; }
    bool loopback() const { return transport == RT_TRANSPORT_RCCL_LOOPBACK; }
    bool threads() const { return transport == RT_TRANSPORT_THREADS; }
    bool via_ipc() const { return transport == RT_TRANSPORT_IPC; }
    // the mailbox transports: every ncclSend/ncclRecv pair is a copy matched through posts
    bool mailbox() const { return threads() || via_ipc(); }
    // the frame goes through an exchange between ranks (a communicator with several ranks or
    // the root's band to itself, or a mailbox); COPY writes the root's frame directly
    bool gathers() const { return (rccl() && (nranks > 1 || loopback())) || mailbox(); }
};

namespace {

struct DevGuard {  // the caller's current device is restored on every return path
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DevGuard(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) err = hipSetDevice(d);
    }
    ~DevGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

int hip_err(rt_multi* m, hipError_t e, const char* what) {
    if (m) std::snprintf(m->last_err, sizeof m->last_err, "%s: %s", what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_HIP;
}
int nccl_err(rt_multi* m, ncclResult_t e, const char* what) {
    if (m) std::snprintf(m->last_err, sizeof m->last_err, "%s: %s", what, ncclGetErrorString(e));
    return RT_ERR_COMM;
}
int ctx_err(rt_multi* m, const Rank* k, int st, const char* what) {
    if (m && st != RT_OK)
        std::snprintf(m->last_err, sizeof m->last_err, "%s (rank %d): %s %s", what, k->rank,
                      rt_strerror(st), k->ctx ? rt_last_hip_error(k->ctx) : "");
    return st;
}

/* RT_MULTI_TRACE=1 (diagnostics): report to stderr every runtime call of the frame path
 * that holds the host for more than 100 us (a call that waits for the GPU). */
bool trace_on() {
    static const bool on = [] {
        const char* e = std::getenv("RT_MULTI_TRACE");
        return e && e[0] == '1';
    }();
    return on;
}
struct SlowCall {
    const char* what;
    std::chrono::steady_clock::time_point t0;
    explicit SlowCall(const char* w) : what(w), t0(trace_on() ? std::chrono::steady_clock::now()
                                                                : std::chrono::steady_clock::time_point{}) {}
    ~SlowCall() {
        if (!trace_on()) return;
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        if (us > 100) std::fprintf(stderr, "rt_multi slow call %.0f us: %s\n", us, what);
    }
};

#define MHIP(m, call)                                          \
    do {                                                       \
        SlowCall sc_(#call);                                   \
        hipError_t e_ = (call);                                \
        if (e_ != hipSuccess) return hip_err((m), e_, #call);  \
    } while (0)
/* the per-frame runtime calls; a diagnostic build (RT_DRY_LAUNCH >= 2) skips them */
#ifndef RT_DRY_LAUNCH
#define RT_DRY_LAUNCH 0
#endif
#define MHIPF(m, call)                       \
    do {                                     \
        if (RT_DRY_LAUNCH < 2) MHIP(m, call); \
    } while (0)
#define MNCCL(m, call)                                           \
    do {                                                         \
        SlowCall sc_(#call);                                     \
        ncclResult_t e_ = (call);                                \
        if (e_ != ncclSuccess) return nccl_err((m), e_, #call);  \
    } while (0)

int bpp(int32_t f) { return rt_out_bytes_per_pixel(f); }

/* ---- RT_TRANSPORT_THREADS mailbox ---- */
int hub_timeout_ms() {
    static const int ms = [] {
        const char* e = std::getenv("RT_MULTI_THREADS_TIMEOUT_MS");
        const int v = e ? std::atoi(e) : 0;
        return v > 0 ? v : 30000;
    }();
    return ms;
}
void hub_fail(rt_multi* m) {
    if (!m->hub) return;
    {
        std::lock_guard<std::mutex> lk(m->hub->mu);
        m->hub->failed = true;
    }
    m->hub->cv.notify_all();
}
/* A handle going away: the exchange ends for its peers, and its posts (which name its
 * events) are withdrawn under the lock — a taker enqueues its wait on a post's event while
 * holding the lock (hub_take), so no wait can reach an event after this returns. */
void hub_leave(rt_multi* m) {
    if (!m->hub) return;
    {
        std::lock_guard<std::mutex> lk(m->hub->mu);
        m->hub->failed = true;
        for (auto* mp : {&m->hub->recv, &m->hub->sent})
            for (auto it = mp->begin(); it != mp->end();)
                it = it->second.owner == m ? mp->erase(it) : std::next(it);
    }
    m->hub->cv.notify_all();
}
void hub_put(rt_multi* m, std::map<std::pair<uint64_t, int>, Post> Hub::*box, uint64_t frame, int rank,
             const Post& p) {
    {
        std::lock_guard<std::mutex> lk(m->hub->mu);
        (m->hub.get()->*box)[{frame, rank}] = p;
    }
    m->hub->cv.notify_all();
}
/* Blocks until the peer has posted (frame, rank) into `box`, then takes the post and, if
 * wait_on is set, makes that stream wait on the post's event (still under the lock). */
int hub_take(rt_multi* m, std::map<std::pair<uint64_t, int>, Post> Hub::*box, uint64_t frame, int rank,
             Post* out, const char* what, hipStream_t wait_on) {
    Hub& h = *m->hub;
    std::unique_lock<std::mutex> lk(h.mu);
    auto& mp = h.*box;
    const bool ok = h.cv.wait_for(lk, std::chrono::milliseconds(hub_timeout_ms()), [&] {
        return h.failed || mp.count({frame, rank}) != 0;
    });
    auto it = mp.find({frame, rank});
    if (it == mp.end()) {
        std::snprintf(m->last_err, sizeof m->last_err, "%s (frame %llu, rank %d): %s", what,
                      (unsigned long long)frame, rank,
                      ok ? "a peer handle failed or was destroyed" : "timed out");
        return RT_ERR_COMM;
    }
    *out = it->second;
    mp.erase(it);
    if (wait_on && out->ev) MHIPF(m, hipStreamWaitEvent(wait_on, out->ev, 0));
    return RT_OK;
}

/* ---- RT_TRANSPORT_IPC mailbox (shared memory between processes) ---- */
template <class T>
T ld_acq(const T* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
template <class T>
void st_rel(T* p, T v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

void ipc_fail(rt_multi* m) {
    if (!m->ipc || !m->ipc->sh) return;
    int32_t none = 0;
    (void)__atomic_compare_exchange_n(&m->ipc->sh->failed_rank, &none, m->first_rank + 1, false,
                                      __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
    st_rel(&m->ipc->sh->failed, 1u);
}
bool pid_gone(int32_t pid) { return pid > 0 && ::kill(pid, 0) != 0 && errno == ESRCH; }
/* Polls `ready` (yield first, then 20-us sleeps) until it holds, a handle failed, the peer's
 * process is gone, or ms passes. */
template <class Pred>
int ipc_wait(rt_multi* m, Pred ready, int peer, const char* what, int64_t ms) {
    IpcShared* sh = m->ipc->sh;
    const auto t0 = std::chrono::steady_clock::now();
    for (int it = 0;; it++) {
        if (ready()) return RT_OK;
        const char* why = nullptr;
        if (ld_acq(&sh->failed)) why = "a peer handle failed";
        if (!why && it >= 2048) {
            if ((it & 255) == 0 && peer >= 0 && pid_gone(sh->peer[peer].pid)) why = "the peer's process exited";
            else if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(ms)) why = "timed out";
        }
        if (why) {
            const int32_t fr = ld_acq(&sh->failed_rank);
            std::snprintf(m->last_err, sizeof m->last_err, "%s (peer rank %d): %s%s", what, peer, why,
                          fr > 0 ? (std::string(" (rank ") + std::to_string(fr - 1) + " failed first)").c_str() : "");
            return RT_ERR_COMM;
        }
        if (it < 2048) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}
int ipc_post(rt_multi* m, IpcRing& r, uint64_t& count, const IpcMsg& v, int peer, const char* what) {
    int st = ipc_wait(m, [&] { return count - ld_acq(&r.taken) < (uint64_t)IPC_RING; }, peer, what,
                      hub_timeout_ms());
    if (st != RT_OK) return st;
    IpcMsg& e = r.msg[count % IPC_RING];
    e.frame = v.frame;
    e.bytes = v.bytes;
    e.offset = v.offset;
    e.alloc = v.alloc;
    e.ev = v.ev;
    e.mem = v.mem;
    st_rel(&e.seq, count + 1);
    count++;
    return RT_OK;
}
int ipc_take(rt_multi* m, IpcRing& r, uint64_t& count, uint64_t frame, IpcMsg* out, int peer, const char* what) {
    IpcMsg& e = r.msg[count % IPC_RING];
    const uint64_t want = count + 1;
    int st = ipc_wait(m, [&] { return ld_acq(&e.seq) == want; }, peer, what, hub_timeout_ms());
    if (st != RT_OK) return st;
    out->frame = e.frame;
    out->bytes = e.bytes;
    out->offset = e.offset;
    out->alloc = e.alloc;
    out->ev = e.ev;
    out->mem = e.mem;
    st_rel(&r.taken, want);
    count++;
    if (out->frame != frame || out->ev < 0 || out->ev >= IPC_NEV) {
        std::snprintf(m->last_err, sizeof m->last_err, "%s (peer rank %d): post for frame %llu, expected %llu",
                      what, peer, (unsigned long long)out->frame, (unsigned long long)frame);
        return RT_ERR_COMM;
    }
    return RT_OK;
}
/* Stream-ordered counters in the shared segment (the IPC transport's events): a host
 * function on a stream sets *word = value once the stream's earlier work is done, or holds
 * the stream until *word >= value (a handle's failure, or the transport timeout, releases
 * it: the exchange is broken by then and the frame's contents are not used). */
struct SeqOp {
    uint64_t* word;
    uint64_t value;
    const uint32_t* failed;
    int64_t timeout_ms;
};
void seq_set_fn(void* a) {
    SeqOp* o = static_cast<SeqOp*>(a);
    st_rel(o->word, o->value);
    delete o;
}
void seq_wait_fn(void* a) {
    SeqOp* o = static_cast<SeqOp*>(a);
    const auto t0 = std::chrono::steady_clock::now();
    for (int it = 0; ld_acq(o->word) < o->value && !ld_acq(o->failed); it++) {
        if (it < 4096) {
            std::this_thread::yield();
        } else {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(o->timeout_ms)) break;
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
    delete o;
}
int seq_enqueue(rt_multi* m, hipStream_t st, uint64_t* word, uint64_t value, bool wait) {
    SeqOp* o = new (std::nothrow) SeqOp{word, value, &m->ipc->sh->failed, hub_timeout_ms()};
    if (!o) return RT_ERR_OUT_OF_MEMORY;
    const hipError_t e = hipLaunchHostFunc(st, wait ? seq_wait_fn : seq_set_fn, o);
    if (e != hipSuccess) {
        delete o;
        return hip_err(m, e, "hipLaunchHostFunc");
    }
    return RT_OK;
}

/* A staging buffer of the root that senders write into: hipMalloc'd and exported once; kept
 * until destroy (a peer may still hold the mapping when it grows). */
int ipc_alloc(rt_multi* m, size_t bytes, void** out) {
    *out = nullptr;
    Ipc::Exp e{};
    MHIP(m, hipMalloc(&e.base, bytes));
    e.bytes = bytes;
    e.id = m->ipc->next_id++;
    const hipError_t he = hipIpcGetMemHandle(&e.h, e.base);
    if (he != hipSuccess) {
        (void)hipFree(e.base);
        return hip_err(m, he, "hipIpcGetMemHandle");
    }
    m->ipc->exp.push_back(e);
    *out = e.base;
    return RT_OK;
}

/* The exchange events of a rank by EV_* index. */
hipEvent_t local_ev(Rank* k, int idx) {
    if (idx < EV_SENT) return k->ev_ready[idx - EV_READY];
    if (idx < EV_BSENT) return k->ev_sent[idx - EV_SENT];
    return k->ev_bsent[idx - EV_BSENT];
}

/* ---- the mailbox transports' four operations (THREADS: the in-process Hub; IPC: rings) ---- */
/* Root: rank g's part of `frame` (a frame or a batch's first frame) lands at dst (bytes)
 * once the root's event ev_idx has fired. */
int mbox_post_recv(rt_multi* m, Rank* k, uint64_t frame, int g, char* dst, size_t bytes, int ev_idx) {
    if (m->threads()) {
        Post p;
        p.dst = dst;
        p.device = k->device;
        p.bytes = bytes;
        p.ev = local_ev(k, ev_idx);
        p.owner = m;
        hub_put(m, &Hub::recv, frame, g, p);
        return RT_OK;
    }
    Ipc& x = *m->ipc;
    const Ipc::Exp* a = nullptr;
    for (const auto& e : x.exp)
        if (dst >= static_cast<char*>(e.base) && dst + bytes <= static_cast<char*>(e.base) + e.bytes) a = &e;
    if (!a) {
        std::snprintf(m->last_err, sizeof m->last_err, "IPC: rank %d's destination is not an exported buffer", g);
        return RT_ERR_COMM;
    }
    IpcMsg v{};
    v.frame = frame;
    v.bytes = bytes;
    v.offset = (uint64_t)(dst - static_cast<char*>(a->base));
    v.alloc = a->id;
    v.ev = ev_idx;
    v.mem = a->h;
    // "ready" for this post once the root's comm stream (where ev_idx was recorded) is here
    const int st = seq_enqueue(m, k->comm_stream, &x.sh->peer[g].ready, x.nrecv[g] + 1, false);
    if (st != RT_OK) return st;
    return ipc_post(m, x.sh->peer[g].recv, x.nrecv[g], v, g, "posting a receive");
}
/* Sender: where this rank's part of `frame` goes (*dst on device *dev); `st` waits until it
 * may be written. */
int mbox_take_recv(rt_multi* m, Rank* k, uint64_t frame, size_t bytes, hipStream_t st, char** dst, int* dev) {
    if (m->threads()) {
        Post p;
        const int e = hub_take(m, &Hub::recv, frame, k->rank, &p, "waiting for the root's receive", st);
        if (e != RT_OK) return e;
        if (p.bytes != bytes) {
            std::snprintf(m->last_err, sizeof m->last_err, "rank %d: the root expects %zu bytes, the part has %zu",
                          k->rank, p.bytes, bytes);
            return RT_ERR_COMM;
        }
        *dst = static_cast<char*>(p.dst);
        *dev = p.device;
        return RT_OK;
    }
    Ipc& x = *m->ipc;
    IpcMsg v{};
    int e = ipc_take(m, x.sh->peer[k->rank].recv, x.nrecv_taken, frame, &v, 0, "waiting for the root's receive");
    if (e != RT_OK) return e;
    if (v.bytes != bytes) {
        std::snprintf(m->last_err, sizeof m->last_err, "rank %d: the root expects %llu bytes, the part has %zu",
                      k->rank, (unsigned long long)v.bytes, bytes);
        return RT_ERR_COMM;
    }
    auto it = x.opened.find(v.alloc);
    if (it == x.opened.end()) {
        void* p = nullptr;
        MHIP(m, hipIpcOpenMemHandle(&p, v.mem, hipIpcMemLazyEnablePeerAccess));
        it = x.opened.emplace(v.alloc, p).first;
    }
    *dst = static_cast<char*>(it->second) + v.offset;
    *dev = k->device;
    // the stream waits for the root's "ready" of this post (ipc_take advanced the count)
    return seq_enqueue(m, st, &x.sh->peer[k->rank].ready, x.nrecv_taken, true);
}
/* Sender: this rank's copy of `frame`'s part is complete once its event ev_idx fires. */
int mbox_post_sent(rt_multi* m, Rank* k, uint64_t frame, int ev_idx) {
    if (m->threads()) {
        Post p;
        p.ev = local_ev(k, ev_idx);
        p.owner = m;
        hub_put(m, &Hub::sent, frame, k->rank, p);
        return RT_OK;
    }
    Ipc& x = *m->ipc;
    IpcMsg v{};
    v.frame = frame;
    v.ev = ev_idx;
    // "sent" for this post once this rank's comm stream (its copy) is here
    const int st = seq_enqueue(m, k->comm_stream, &x.sh->peer[k->rank].sent, x.nsent_posted + 1, false);
    if (st != RT_OK) return st;
    return ipc_post(m, x.sh->peer[k->rank].sent_ring, x.nsent_posted, v, 0, "posting a send");
}
/* Root: `st` waits until rank g's part of `frame` has landed. */
int mbox_take_sent(rt_multi* m, Rank* k, uint64_t frame, int g, hipStream_t st) {
    (void)k;
    if (m->threads()) {
        Post p;
        return hub_take(m, &Hub::sent, frame, g, &p, "waiting for a part's copy", st);
    }
    Ipc& x = *m->ipc;
    IpcMsg v{};
    const int e = ipc_take(m, x.sh->peer[g].sent_ring, x.nsent[g], frame, &v, g, "waiting for a part's copy");
    if (e != RT_OK) return e;
    return seq_enqueue(m, st, &x.sh->peer[g].sent, x.nsent[g], true);
}
/* A sender's copy into the destination mbox_take_recv returned. */
int mbox_copy(rt_multi* m, Rank* k, char* dst, int dev, const void* src, size_t bytes, hipStream_t st) {
    if (m->threads()) MHIPF(m, hipMemcpyPeerAsync(dst, dev, src, k->device, bytes, st));
    else MHIPF(m, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
    return RT_OK;
}

/* RT_OPT_MULTI_FAULT (test hook): this frame fails here, once this rank's part of the
 * exchange has been queued. */
bool injected(rt_multi* m) {
    if (!m->fault_next) return false;
    m->fault_next = false;
    std::snprintf(m->last_err, sizeof m->last_err,
                  "injected fault (rank %d) after its part of the exchange was queued", m->first_rank);
    return true;
}

/* Band buffers of a rank, grown (rarely) to `bytes` each: a non-root rank renders into them
 * on its render streams; the root does too under RT_TRANSPORT_RCCL_LOOPBACK, on the CALLER's
 * stream.  Draining the render and comm streams also covers those caller-stream renders:
 * every one is followed by a comm-stream wait on ev_rendered[s] before its self-send, so the
 * comm stream completes only after them. */
int ensure_bands(rt_multi* m, Rank* k, size_t bytes) {
    if (bytes <= k->band_cap) return RT_OK;
    // nothing in flight may still read or write the old buffers
    for (auto rs : k->render_stream) MHIP(m, hipStreamSynchronize(rs));
    MHIP(m, hipStreamSynchronize(k->comm_stream));
    for (auto& b : k->band) {
        if (b) MHIP(m, hipFree(b));
        b = nullptr;
    }
    k->band_cap = 0;
    for (auto& b : k->band) MHIP(m, hipMalloc(&b, bytes));
    k->band_cap = bytes;
    return RT_OK;
}

/* A rank's rows of the frame: contiguous band (row0, nrows) or interleaved part (nrows). */
struct Part {
    int32_t row0 = 0, nrows = 0;
};
Part part_of(const rt_multi* m, int32_t height, int rank) {
    Part pt;
    if (m->layout == 1 && m->nranks > 1)
        (void)rt_interleaved_rows(height, m->nranks, rank, &pt.nrows);
    else if (m->layout == 2 && m->nranks > 1 &&
             rt_weighted_band_rows(height, m->nranks, rank, m->weights.data(), (int32_t)m->weights.size(),
                                   &pt.row0, &pt.nrows) == RT_OK)
        ;  // weighted bands (equal bands below while the weights do not cover this frame)
    else
        (void)rt_band_rows(height, m->nranks, rank, &pt.row0, &pt.nrows);
    return pt;
}
/* Largest part of any rank (band buffer / staging size in rows). */
int32_t max_part_rows(const rt_multi* m, int32_t height) {
    int32_t mx = 0;
    for (int g = 0; g < m->nranks; g++) mx = std::max(mx, part_of(m, height, g).nrows);
    return mx;
}
/* Interleaved part `part` stored back to back at src -> its rows of the frame (tile rows of
 * TH = rt_tile_rows() pixel rows: a strided 2D copy of the full ones, then the frame's short
 * last tile row if it is this part's). */
int scatter_part(rt_multi* m, char* frame, const char* src, int32_t height, int part,
                 size_t row_bytes, hipStream_t st) {
    const int N = m->nranks, TH = rt_tile_rows(), T = (height + TH - 1) / TH;
    if (part >= T || row_bytes == 0) return RT_OK;
    const int nt = (T - part + N - 1) / N;
    const bool partial = (height % TH) != 0 && ((T - 1) % N) == part;
    const int nfull = nt - (partial ? 1 : 0);
    const size_t tile_bytes = (size_t)TH * row_bytes;
    if (nfull > 0)
        MHIP(m, hipMemcpy2DAsync(frame + (size_t)part * tile_bytes, (size_t)N * tile_bytes, src,
                                 tile_bytes, tile_bytes, (size_t)nfull, hipMemcpyDefault, st));
    if (partial)
        MHIP(m, hipMemcpyAsync(frame + (size_t)(T - 1) * tile_bytes, src + (size_t)nfull * tile_bytes,
                               (size_t)(height % TH) * row_bytes, hipMemcpyDefault, st));
    return RT_OK;
}
/* A rank's rows rendered into `dst` on `st`: contiguous band -> dst + row0 rows (dst is the
 * frame) or back to back (dst is a band buffer); interleaved part -> its frame rows
 * (to_frame) or back to back. */
int render_part(rt_multi* m, Rank* k, const Job& j, const Part& pt, char* dst, bool to_frame,
                hipStream_t st) {
    const rt_camera& cam = *j.cam;
    const size_t row_bytes = (size_t)cam.width * bpp(j.out_format);
    int e;
    if (m->layout == 1 && m->nranks > 1)
        e = rt_render_device_interleaved(k->ctx, &cam, m->nranks, k->rank, j.depth, j.precision,
                                         j.flags, j.out_format, dst, to_frame ? 1 : 0, nullptr, st);
    else
        e = rt_render_device(k->ctx, &cam, pt.row0, pt.nrows, j.depth, j.precision, j.flags,
                             j.out_format, to_frame ? dst + (size_t)pt.row0 * row_bytes : dst,
                             nullptr, st);
    return ctx_err(m, k, e, "rt_render_device");
}

/* One rank's share of one frame (see the file comment).  Runs on the caller's thread for
 * the first local rank and on the rank's worker thread for the others. */
int enqueue_rank(rt_multi* m, Rank* k, const Job& j) {
    DevGuard dg(k->device);
    MHIP(m, dg.err);
    const rt_camera& cam = *j.cam;
    const size_t row_bytes = (size_t)cam.width * bpp(j.out_format);
    const bool inter = m->layout == 1 && m->nranks > 1;
    const Part pt = part_of(m, cam.height, k->rank);
    const int32_t nrows = pt.nrows;
    int st = RT_OK;
    const int s = j.slot;
    if (k->rank == 0) {
        const bool lb = m->loopback() && nrows > 0 && row_bytes > 0;
        if (lb) {
            // RT_TRANSPORT_RCCL_LOOPBACK: the root's rows into its band slot on the caller's
            // stream (once the slot's previous self-send has completed), sent to itself below
            st = ensure_bands(m, k, (size_t)max_part_rows(m, cam.height) * row_bytes);
            if (st != RT_OK) return st;
            MHIPF(m, hipStreamWaitEvent(j.stream, k->ev_sent[s], 0));
            SlowCall sc_("rt_render_device (root, loopback)");
            st = render_part(m, k, j, pt, static_cast<char*>(k->band[s]), false, j.stream);
            if (st != RT_OK) return st;
            MHIPF(m, hipEventRecord(k->ev_rendered[s], j.stream));
        } else if (nrows > 0) {
            // the root's rows, in place in the frame, on the caller's stream
            SlowCall sc_("rt_render_device (root)");
            st = render_part(m, k, j, pt, j.d_frame, true, j.stream);
            if (st != RT_OK) return st;
        }
        if (m->gathers()) {
            m->queued.store(true, std::memory_order_relaxed);
            const size_t part_bytes = (size_t)max_part_rows(m, cam.height) * row_bytes;
            // parts land in staging (then go to their rows on the comm stream): interleaved
            // parts always; every part under IPC (senders write only exported buffers)
            const bool staged = inter || m->via_ipc();
            if (staged && part_bytes * m->nranks > k->staging_cap) {
                // grow (rare): the comm stream may still scatter from the old buffers
                MHIP(m, hipStreamSynchronize(k->comm_stream));
                for (auto& b : k->staging) {
                    if (b && !m->via_ipc()) MHIP(m, hipFree(b));  // IPC: kept until destroy
                    b = nullptr;
                }
                k->staging_cap = 0;
                for (auto& b : k->staging) {
                    if (m->via_ipc()) {
                        st = ipc_alloc(m, part_bytes * m->nranks, &b);
                        if (st != RT_OK) return st;
                    } else {
                        MHIP(m, hipMalloc(&b, part_bytes * m->nranks));
                    }
                }
                k->staging_cap = part_bytes * m->nranks;
            }
            MHIPF(m, hipStreamWaitEvent(k->comm_stream, j.ev_in, 0));
            if (m->mailbox()) {
                // the mailbox's receives: post where every part lands (after ev_ready: the
                // caller's earlier work on the frame is done), then wait on each part's copy
                MHIPF(m, hipEventRecord(k->ev_ready[s], k->comm_stream));
                for (int g = 1; g < m->nranks; g++) {
                    const Part pg = part_of(m, cam.height, g);
                    if (pg.nrows <= 0 || row_bytes == 0) continue;
                    char* dst = staged ? static_cast<char*>(k->staging[s]) + (size_t)g * part_bytes
                                       : j.d_frame + (size_t)pg.row0 * row_bytes;
                    st = mbox_post_recv(m, k, m->frame, g, dst, (size_t)pg.nrows * row_bytes, EV_READY + s);
                    if (st != RT_OK) return st;
                }
                if (injected(m)) return RT_ERR_HIP;
                for (int g = 1; g < m->nranks; g++) {
                    const Part pg = part_of(m, cam.height, g);
                    if (pg.nrows <= 0 || row_bytes == 0) continue;
                    st = mbox_take_sent(m, k, m->frame, g, k->comm_stream);
                    if (st != RT_OK) return st;
                }
                if (staged)
                    for (int g = 1; g < m->nranks; g++) {
                        const Part pg = part_of(m, cam.height, g);
                        const char* src = static_cast<char*>(k->staging[s]) + (size_t)g * part_bytes;
                        if (inter)
                            st = scatter_part(m, j.d_frame, src, cam.height, g, row_bytes, k->comm_stream);
                        else if (pg.nrows > 0 && row_bytes > 0)
                            MHIPF(m, hipMemcpyAsync(j.d_frame + (size_t)pg.row0 * row_bytes, src,
                                                    (size_t)pg.nrows * row_bytes, hipMemcpyDeviceToDevice,
                                                    k->comm_stream));
                        if (st != RT_OK) return st;
                    }
                MHIPF(m, hipEventRecord(k->ev_done, k->comm_stream));
                return RT_OK;
            }
            if (lb) MHIPF(m, hipStreamWaitEvent(k->comm_stream, k->ev_rendered[s], 0));
            MNCCL(m, ncclGroupStart());
            if (lb) {
                const size_t bytes = (size_t)nrows * row_bytes;
                char* dst = inter ? static_cast<char*>(k->staging[s]) : j.d_frame + (size_t)pt.row0 * row_bytes;
                ncclResult_t e = ncclSend(k->band[s], bytes, ncclUint8, 0, k->comm, k->comm_stream);
                if (e == ncclSuccess) e = ncclRecv(dst, bytes, ncclUint8, 0, k->comm, k->comm_stream);
                if (e != ncclSuccess) {
                    (void)ncclGroupEnd();
                    return nccl_err(m, e, "ncclSend/ncclRecv (root to itself)");
                }
            }
            for (int g = 1; g < m->nranks; g++) {
                const Part pg = part_of(m, cam.height, g);
                if (pg.nrows <= 0 || row_bytes == 0) continue;
                char* dst = inter ? static_cast<char*>(k->staging[s]) + (size_t)g * part_bytes
                                  : j.d_frame + (size_t)pg.row0 * row_bytes;
                const ncclResult_t e = ncclRecv(dst, (size_t)pg.nrows * row_bytes, ncclUint8, g,
                                                k->comm, k->comm_stream);
                if (e != ncclSuccess) {
                    (void)ncclGroupEnd();
                    return nccl_err(m, e, "ncclRecv");
                }
            }
            MNCCL(m, ncclGroupEnd());
            if (injected(m)) return RT_ERR_HIP;
            if (inter)
                for (int g = lb ? 0 : 1; g < m->nranks; g++) {
                    st = scatter_part(m, j.d_frame, static_cast<char*>(k->staging[s]) + (size_t)g * part_bytes,
                                      cam.height, g, row_bytes, k->comm_stream);
                    if (st != RT_OK) return st;
                }
            MHIPF(m, hipEventRecord(k->ev_done, k->comm_stream));
            if (lb) MHIPF(m, hipEventRecord(k->ev_sent[s], k->comm_stream));  // slot s free again
        }
        return RT_OK;
    }
    const size_t bytes = (size_t)nrows * row_bytes;
    if (bytes == 0) return RT_OK;  // an empty band (height < nranks): nothing to render or send
    st = ensure_bands(m, k, (size_t)max_part_rows(m, cam.height) * row_bytes);
    if (st != RT_OK) return st;
    // band buffer `s` is free once the send of frame k - slots has completed
    MHIPF(m, hipStreamWaitEvent(k->render_stream[s], k->ev_sent[s], 0));
    {
        SlowCall sc_("rt_render_device (band)");
        st = render_part(m, k, j, pt, static_cast<char*>(k->band[s]), false, k->render_stream[s]);
    }
    if (st != RT_OK) return st;
    MHIPF(m, hipEventRecord(k->ev_rendered[s], k->render_stream[s]));
    MHIPF(m, hipStreamWaitEvent(k->comm_stream, k->ev_rendered[s], 0));
    m->queued.store(true, std::memory_order_relaxed);
    if (m->rccl()) {
        MNCCL(m, ncclSend(k->band[s], bytes, ncclUint8, 0, k->comm, k->comm_stream));
        if (injected(m)) return RT_ERR_HIP;
    } else if (m->mailbox()) {
        // the mailbox's send: where the root wants this part, once it may be written
        char* dst = nullptr;
        int ddev = 0;
        st = mbox_take_recv(m, k, m->frame, bytes, k->comm_stream, &dst, &ddev);
        if (st != RT_OK) return st;
        st = mbox_copy(m, k, dst, ddev, k->band[s], bytes, k->comm_stream);
        if (st != RT_OK) return st;
        MHIPF(m, hipEventRecord(k->ev_sent[s], k->comm_stream));
        st = mbox_post_sent(m, k, m->frame, EV_SENT + s);
        if (st != RT_OK) return st;
        if (injected(m)) return RT_ERR_HIP;
    } else {
        // the root's rows may still be read by the caller's earlier work on the frame buffer
        MHIPF(m, hipStreamWaitEvent(k->comm_stream, j.ev_in, 0));
        if (inter) {
            st = scatter_part(m, j.d_frame, static_cast<const char*>(k->band[s]), cam.height, k->rank,
                              row_bytes, k->comm_stream);
            if (st != RT_OK) return st;
        } else {
            MHIPF(m, hipMemcpyPeerAsync(j.d_frame + (size_t)pt.row0 * row_bytes, m->r[0]->device, k->band[s],
                                       k->device, bytes, k->comm_stream));
        }
    }
    if (!m->mailbox()) MHIPF(m, hipEventRecord(k->ev_sent[s], k->comm_stream));  // mailbox: above
    // a process without the root: work the caller enqueues later on its stream (on this
    // rank's device) follows the band's send
    if (j.stream && !m->has_root())
        MHIPF(m, hipStreamWaitEvent(j.stream, k->ev_sent[s], 0));
    return RT_OK;
}

/* ---- batched gather (RT_OPT_MULTI_BATCH) ----
 * A batch of kb frames is one exchange: every sender renders its band of the kb frames back
 * to back into bbuf (the ctx's own frame loop, with its host pipeline, round-robin over its
 * render streams) and sends the kb bands in ONE ncclSend; the root renders its rows of the kb frames in place
 * on the caller's streams, receives every rank's kb bands into bstage in ONE group, and
 * copies them into the frames' rows with one scatter kernel.  Two batch slots: batch b + 1
 * renders while batch b is in flight.  Per frame that is one launch plus 1/kb of the
 * exchange's calls (events, RCCL), which cost more than a 1/8 band's kernel when paid per
 * frame (tools/nonroot_host_cost.py). */
struct ScatterSeg {
    const char* src;
    char* dst;
    uint64_t bytes;
};
constexpr int SCATTER_MAX = 128;  // segments per launch (kernel arguments ~3 KB)
struct ScatterArgs {
    int32_t nseg, vec16;
    ScatterSeg seg[SCATTER_MAX];
};
/* Segment blockIdx.y: bytes from src to dst, 16 B per lane when every segment allows it. */
__global__ void __launch_bounds__(256) k_scatter_parts(ScatterArgs a) {
    const ScatterSeg sg = a.seg[blockIdx.y];
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a.vec16) {
        const uint4* src = reinterpret_cast<const uint4*>(sg.src);
        uint4* dst = reinterpret_cast<uint4*>(sg.dst);
        for (size_t i = i0; i < sg.bytes / 16; i += stride) dst[i] = src[i];
    } else {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(sg.src);
        uint32_t* dst = reinterpret_cast<uint32_t*>(sg.dst);
        for (size_t i = i0; i < sg.bytes / 4; i += stride) dst[i] = src[i];
    }
}
/* The segments in order (those of frame fidx[j] land in frames[fidx[j]]), one launch per
 * run in which no frame buffer repeats — a batch that cycles over fewer buffers than frames
 * lands its frames in frame order, as frame-by-frame gathers would — and at most
 * SCATTER_MAX segments. */
int scatter_segments(rt_multi* m, const std::vector<ScatterSeg>& segs, const std::vector<int>& fidx,
                     char* const* frames, hipStream_t st) {
    size_t i = 0;
    while (i < segs.size()) {
        ScatterArgs a{};
        std::vector<char*> used;
        size_t maxb = 0;
        bool vec = true;
        size_t j = i;
        for (; j < segs.size() && a.nseg < SCATTER_MAX; j++) {
            if (j == i || fidx[j] != fidx[j - 1]) {  // the first segment of a frame
                char* fb = frames[fidx[j]];
                if (std::find(used.begin(), used.end(), fb) != used.end()) break;
                used.push_back(fb);
            }
            a.seg[a.nseg++] = segs[j];
            maxb = std::max<size_t>(maxb, segs[j].bytes);
            vec = vec && ((reinterpret_cast<uintptr_t>(segs[j].src) | reinterpret_cast<uintptr_t>(segs[j].dst) |
                           (uintptr_t)segs[j].bytes) & 15) == 0;
        }
        a.vec16 = vec ? 1 : 0;
        const size_t units = vec ? maxb / 16 : maxb / 4;
        const unsigned gx = (unsigned)std::max<size_t>(1, std::min<size_t>(256, (units + 255) / 256));
        hipLaunchKernelGGL(k_scatter_parts, dim3(gx, (unsigned)a.nseg), dim3(256), 0, st, a);
        MHIP(m, hipGetLastError());
        i = j;
    }
    return RT_OK;
}
/* Batch parameters shared by the roles. */
struct BatchJob {
    const rt_camera* cams = nullptr;  // kb cameras (equal sizes)
    int kb = 0, bs = 0;
    int32_t depth = 0, precision = 0, out_format = 0;
    uint32_t flags = 0;
};
/* A sender's batch (a non-root rank; the root itself under RT_TRANSPORT_RCCL_LOOPBACK, self:
 * render only, its send is in the root's group). */
int batch_send(rt_multi* m, Rank* k, const BatchJob& b, bool self) {
    const rt_camera& cam = b.cams[0];
    const size_t row_bytes = (size_t)cam.width * bpp(b.out_format);
    const Part pt = part_of(m, cam.height, k->rank);
    const size_t bytes = (size_t)pt.nrows * row_bytes;
    if (bytes == 0) return RT_OK;  // an empty band: nothing to render or send (the root posts none)
    const size_t need = (size_t)b.kb * (size_t)max_part_rows(m, cam.height) * row_bytes;
    if (need > k->bbuf_cap) {  // grow (rare): nothing in flight may use the old buffers
        for (auto rs : k->render_stream) MHIP(m, hipStreamSynchronize(rs));
        MHIP(m, hipStreamSynchronize(k->comm_stream));
        for (auto& p : k->bbuf) {
            if (p) MHIP(m, hipFree(p));
            p = nullptr;
        }
        k->bbuf_cap = 0;
        for (auto& p : k->bbuf) MHIP(m, hipMalloc(&p, need));
        k->bbuf_cap = need;
    }
    // the batch's frames round-robin over RT_OPT_MULTI_FRAMES render streams, so a small
    // band's long last waves overlap the next frames' (one stream would run them one after
    // another), each stream first waiting until this slot's last send is done
    // (RT_OPT_FRAME_BATCH = fb: blocks of fb consecutive frames per stream instead, over
    // ceil(kb / fb) streams, so the ctx launches each block as one grid)
    const int fb = m->frame_batch;
    const int S = fb > 1 ? std::max(1, std::min(m->slots, (b.kb + fb - 1) / fb))
                         : std::max(1, std::min(m->slots, b.kb));
    for (int j = 0; j < S; j++) MHIPF(m, hipStreamWaitEvent(k->render_stream[j], k->ev_bsent[b.bs], 0));
    void* sts[RT_MULTI_BATCH_MAX];  // frame i's stream
    for (int i = 0; i < b.kb; i++)
        sts[i] = k->render_stream[fb > 1 ? std::min(i / fb, S - 1) : i % S];
    void* outs[RT_MULTI_BATCH_MAX];
    for (int i = 0; i < b.kb; i++) outs[i] = static_cast<char*>(k->bbuf[b.bs]) + (size_t)i * bytes;
    {
        SlowCall sc_("rt_render_device_frames (batch)");
        const int e = rt_render_device_frames(k->ctx, b.cams, b.kb, pt.row0, pt.nrows, b.depth, b.precision,
                                              b.flags, b.out_format, outs, b.kb, sts, b.kb, b.kb);
        if (e != RT_OK) return ctx_err(m, k, e, "rt_render_device_frames (batch)");
    }
    for (int j = 0; j < S; j++) {  // the send follows every stream's frames
        MHIPF(m, hipEventRecord(k->ev_brend[b.bs][j], k->render_stream[j]));
        MHIPF(m, hipStreamWaitEvent(k->comm_stream, k->ev_brend[b.bs][j], 0));
    }
    if (self) return RT_OK;
    m->queued.store(true, std::memory_order_relaxed);
    const size_t total = (size_t)b.kb * bytes;
    if (m->rccl()) {
        MNCCL(m, ncclSend(k->bbuf[b.bs], total, ncclUint8, 0, k->comm, k->comm_stream));
        MHIPF(m, hipEventRecord(k->ev_bsent[b.bs], k->comm_stream));
        return injected(m) ? RT_ERR_HIP : RT_OK;
    }
    // the mailbox's send, keyed by the batch's first frame
    char* dst = nullptr;
    int ddev = 0;
    int st = mbox_take_recv(m, k, m->frame, total, k->comm_stream, &dst, &ddev);
    if (st != RT_OK) return st;
    st = mbox_copy(m, k, dst, ddev, k->bbuf[b.bs], total, k->comm_stream);
    if (st != RT_OK) return st;
    MHIPF(m, hipEventRecord(k->ev_bsent[b.bs], k->comm_stream));
    st = mbox_post_sent(m, k, m->frame, EV_BSENT + b.bs);
    if (st != RT_OK) return st;
    return injected(m) ? RT_ERR_HIP : RT_OK;
}
/* The root's batch: frames[i] / sts[i] = frame i's buffer and caller stream (distinct streams
 * listed in uniq, at most RT_MULTI_SLOTS; the kb buffers distinct, checked by the caller). */
int batch_root(rt_multi* m, Rank* k, const BatchJob& b, char* const* frames, hipStream_t const* sts,
               const std::vector<hipStream_t>& uniq) {
    const rt_camera& cam = b.cams[0];
    const size_t row_bytes = (size_t)cam.width * bpp(b.out_format);
    const int N = m->nranks;
    const bool lb = m->loopback();
    // a frame buffer of an earlier batch is rendered into again only once that batch's
    // scatter has completed, so each frame is whole in its buffer between its batch's end and
    // the next render into that buffer.  The previous batch's buffers wait on its done event;
    // the one before's on ev_bdone[bs], which still holds that batch's record (and the comm
    // stream runs batches in order, so it also covers every older one).
    // RT_OPT_FRAME_BATCH = fb: the root's rows of each block of fb consecutive frames are
    // rendered on the block's first frame's stream (one launch); a frame of another caller
    // stream is ordered around it (its stream's earlier work before, its later work after)
    const int fb = m->frame_batch;
    hipStream_t rs[RT_MULTI_BATCH_MAX];
    bool cross = false;
    for (int i = 0; i < b.kb; i++) {
        rs[i] = fb > 1 ? sts[(i / fb) * fb] : sts[i];
        cross = cross || rs[i] != sts[i];
    }
    std::vector<hipStream_t> rset;  // the streams that render
    for (int i = 0; i < b.kb; i++)
        if (std::find(rset.begin(), rset.end(), rs[i]) == rset.end()) rset.push_back(rs[i]);
    {
        std::vector<std::pair<hipStream_t, int>> waits;
        const int prev = 1 - b.bs;
        for (int i = 0; i < b.kb; i++) {
            int slot = -1;
            if (std::find(m->batch_bufs[prev].begin(), m->batch_bufs[prev].end(), frames[i]) !=
                m->batch_bufs[prev].end())
                slot = prev;
            else if (std::find(m->batch_bufs[b.bs].begin(), m->batch_bufs[b.bs].end(), frames[i]) !=
                     m->batch_bufs[b.bs].end())
                slot = b.bs;
            if (slot >= 0 && std::find(waits.begin(), waits.end(), std::make_pair(rs[i], slot)) == waits.end())
                waits.emplace_back(rs[i], slot);
        }
        for (const auto& w : waits) MHIPF(m, hipStreamWaitEvent(w.first, k->ev_bdone[w.second], 0));
    }
    // the scatter overwrites rows of frames that the caller's earlier work may still read
    for (size_t u = 0; u < uniq.size(); u++) {
        MHIPF(m, hipEventRecord(m->ev_in[u], uniq[u]));
        MHIPF(m, hipStreamWaitEvent(k->comm_stream, m->ev_in[u], 0));
        // the root's rows of a frame of stream u rendered on another stream follow u's earlier work
        if (cross)
            for (hipStream_t r : rset)
                if (r != uniq[u]) MHIPF(m, hipStreamWaitEvent(r, m->ev_in[u], 0));
    }
    const Part p0 = part_of(m, cam.height, 0);
    int st = RT_OK;
    if (lb) {
        st = batch_send(m, k, b, true);
    } else if (p0.nrows > 0 && row_bytes > 0) {
        void* outs[RT_MULTI_BATCH_MAX];
        void* ss[RT_MULTI_BATCH_MAX];
        for (int i = 0; i < b.kb; i++) {
            outs[i] = frames[i] + (size_t)p0.row0 * row_bytes;
            ss[i] = rs[i];
        }
        SlowCall sc_("rt_render_device_frames (root batch)");
        const int e = rt_render_device_frames(k->ctx, b.cams, b.kb, p0.row0, p0.nrows, b.depth, b.precision,
                                              b.flags, b.out_format, outs, b.kb, ss, b.kb, b.kb);
        st = ctx_err(m, k, e, "rt_render_device_frames (root batch)");
        if (st == RT_OK && cross) {
            // work the caller enqueues on the batch's streams sees their frames' rows
            for (size_t j = 0; j < rset.size() && j < (size_t)RT_MULTI_SLOTS; j++) {
                MHIPF(m, hipEventRecord(k->ev_rows[j], rset[j]));
                for (hipStream_t u : uniq)
                    if (u != rset[j]) MHIPF(m, hipStreamWaitEvent(u, k->ev_rows[j], 0));
            }
        }
    }
    if (st != RT_OK) return st;
    m->batch_bufs[b.bs].assign(frames, frames + b.kb);
    // every sender's kb parts back to back in bstage[bs]
    std::vector<size_t> off((size_t)N, 0), pb((size_t)N, 0);
    std::vector<Part> parts((size_t)N);
    size_t total = 0;
    for (int g = lb ? 0 : 1; g < N; g++) {
        parts[g] = part_of(m, cam.height, g);
        pb[g] = (size_t)parts[g].nrows * row_bytes;
        off[g] = total;
        total += (size_t)b.kb * pb[g];
    }
    if (total == 0) {
        MHIPF(m, hipEventRecord(k->ev_done, k->comm_stream));
        MHIPF(m, hipEventRecord(k->ev_bdone[b.bs], k->comm_stream));
        return RT_OK;
    }
    if (total > k->bstage_cap) {  // grow (rare): the comm stream may still scatter from them
        MHIP(m, hipStreamSynchronize(k->comm_stream));
        for (auto& p : k->bstage) {
            if (p && !m->via_ipc()) MHIP(m, hipFree(p));  // IPC: kept until destroy
            p = nullptr;
        }
        k->bstage_cap = 0;
        for (auto& p : k->bstage) {
            if (m->via_ipc()) {
                st = ipc_alloc(m, total, &p);
                if (st != RT_OK) return st;
            } else {
                MHIP(m, hipMalloc(&p, total));
            }
        }
        k->bstage_cap = total;
    }
    char* stage = static_cast<char*>(k->bstage[b.bs]);
    m->queued.store(true, std::memory_order_relaxed);
    if (m->mailbox()) {
        MHIPF(m, hipEventRecord(k->ev_ready[b.bs], k->comm_stream));
        for (int g = 1; g < N; g++) {
            if (pb[g] == 0) continue;
            st = mbox_post_recv(m, k, m->frame, g, stage + off[g], (size_t)b.kb * pb[g], EV_READY + b.bs);
            if (st != RT_OK) return st;
        }
        if (injected(m)) return RT_ERR_HIP;
        for (int g = 1; g < N; g++) {
            if (pb[g] == 0) continue;
            st = mbox_take_sent(m, k, m->frame, g, k->comm_stream);
            if (st != RT_OK) return st;
        }
    } else {
        MNCCL(m, ncclGroupStart());
        for (int g = lb ? 0 : 1; g < N; g++) {
            if (pb[g] == 0) continue;
            ncclResult_t e = ncclSuccess;
            if (g == 0) e = ncclSend(k->bbuf[b.bs], (size_t)b.kb * pb[0], ncclUint8, 0, k->comm, k->comm_stream);
            if (e == ncclSuccess)
                e = ncclRecv(stage + off[g], (size_t)b.kb * pb[g], ncclUint8, g, k->comm, k->comm_stream);
            if (e != ncclSuccess) {
                (void)ncclGroupEnd();
                return nccl_err(m, e, "ncclRecv (batch)");
            }
        }
        MNCCL(m, ncclGroupEnd());
        if (injected(m)) return RT_ERR_HIP;
    }
    std::vector<ScatterSeg> segs;
    std::vector<int> fidx;
    for (int i = 0; i < b.kb; i++)
        for (int g = lb ? 0 : 1; g < N; g++) {
            if (pb[g] == 0) continue;
            segs.push_back({stage + off[g] + (size_t)i * pb[g], frames[i] + (size_t)parts[g].row0 * row_bytes,
                            (uint64_t)pb[g]});
            fidx.push_back(i);
        }
    st = scatter_segments(m, segs, fidx, frames, k->comm_stream);
    if (st != RT_OK) return st;
    MHIPF(m, hipEventRecord(k->ev_done, k->comm_stream));
    MHIPF(m, hipEventRecord(k->ev_bdone[b.bs], k->comm_stream));
    if (lb) MHIPF(m, hipEventRecord(k->ev_bsent[b.bs], k->comm_stream));  // bbuf slot free again
    return RT_OK;
}

void worker_main(rt_multi* m, Rank* k) {
    uint64_t seen = 0;
    for (;;) {
        // spin briefly (a frame loop posts every few tens of microseconds), then sleep
        uint64_t p = k->posted.load(std::memory_order_acquire);
        for (int it = 0; p == seen && it < 4096; it++) {
            std::this_thread::yield();
            p = k->posted.load(std::memory_order_acquire);
        }
        if (p == seen) {
            std::unique_lock<std::mutex> lk(k->mu);
            k->cv.wait(lk, [&] { return k->quit || k->posted.load(std::memory_order_acquire) != seen; });
            if (k->quit) return;
            p = k->posted.load(std::memory_order_acquire);
        }
        seen = p;
        k->status = enqueue_rank(m, k, k->job);
        k->finished.store(seen, std::memory_order_release);
    }
}

void destroy_rank(Rank* k, bool abort_comm) {
    if (k->th.joinable()) {
        {
            std::lock_guard<std::mutex> lk(k->mu);
            k->quit = true;
        }
        k->cv.notify_one();
        k->th.join();
    }
    DevGuard dg(k->device);
    for (auto rs : k->render_stream)
        if (rs) (void)hipStreamSynchronize(rs);
    if (k->comm_stream) (void)hipStreamSynchronize(k->comm_stream);
    if (k->comm) (void)(abort_comm ? ncclCommAbort(k->comm) : ncclCommDestroy(k->comm));
    for (auto& b : k->band)
        if (b) (void)hipFree(b);
    for (int s = 0; s < RT_MULTI_SLOTS; s++) {
        if (k->ev_rendered[s]) (void)hipEventDestroy(k->ev_rendered[s]);
        if (k->ev_sent[s]) (void)hipEventDestroy(k->ev_sent[s]);
    }
    if (k->ev_done) (void)hipEventDestroy(k->ev_done);
    for (int b = 0; b < 2; b++) {
        for (auto e : k->ev_brend[b])
            if (e) (void)hipEventDestroy(e);
        if (k->ev_bsent[b]) (void)hipEventDestroy(k->ev_bsent[b]);
        if (k->ev_bdone[b]) (void)hipEventDestroy(k->ev_bdone[b]);
        if (k->bbuf[b]) (void)hipFree(k->bbuf[b]);
        if (k->bstage[b]) (void)hipFree(k->bstage[b]);
    }
    for (auto e : k->ev_drain)
        if (e) (void)hipEventDestroy(e);
    for (auto e : k->ev_rows)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : k->ev_ready)
        if (e) (void)hipEventDestroy(e);
    for (auto& b : k->staging)
        if (b) (void)hipFree(b);
    for (auto rs : k->render_stream)
        if (rs) (void)hipStreamDestroy(rs);
    if (k->comm_stream) (void)hipStreamDestroy(k->comm_stream);
    if (k->ctx) (void)rt_ctx_destroy(k->ctx);
    delete k;
}

/* A tile-row weight both weight entry points accept: finite and >= 0 (NaN, negatives and inf
 * rejected, so prefix sums and band cuts stay finite). */
bool valid_weight(float w) { return w >= 0.0f && w <= 3.0e38f; }

int check_args(const rt_multi* m, const rt_camera* cam, int32_t depth, int32_t precision,
               int32_t out_format) {
    if (!m || !cam) return RT_ERR_INVALID_ARG;
    if (cam->width < 0 || cam->height < 0 || depth < 0) return RT_ERR_INVALID_ARG;
    if (depth > rt_max_depth()) return RT_ERR_UNSUPPORTED;
    if (precision < RT_PREC_F64 || precision > RT_PREC_PATH64) return RT_ERR_INVALID_ARG;
    if (bpp(out_format) == 0) return RT_ERR_INVALID_ARG;
    return RT_OK;
}

/* A frame (or batch) failed after its arguments were checked (checks every rank makes alike
 * come first and leave the rt_multi usable).  With ranks in other processes (nlocal <
 * nranks) the peers queue their parts of the exchange whatever this process did — a
 * failure only here (a HIP error on this rank's band, its scene missing) leaves them out of
 * step — so the exchange is broken; the mailbox transports also end it for their peers
 * (their waits give up).  With every rank in this process, only a failure after a local rank
 * queued its part breaks it. */
void mark_failed(rt_multi* m) {
    if (m->mailbox()) {
        m->broken = true;
        hub_fail(m);
        ipc_fail(m);
    } else if (m->gathers() && (m->nlocal < m->nranks || m->queued.load(std::memory_order_relaxed))) {
        m->broken = true;
    }
}

/* ---- RT_TRANSPORT_IPC setup and teardown ---- */
/* Opens (or creates) the id's segment and waits until every rank has joined. */
int ipc_create(rt_multi* m, const uint8_t* id) {
    m->ipc.reset(new (std::nothrow) Ipc());
    if (!m->ipc) return RT_ERR_OUT_OF_MEMORY;
    Ipc& x = *m->ipc;
    char name[64];
    int n = std::snprintf(name, sizeof name, "/rtamd-ipc-");
    for (int i = 0; i < 16; i++) n += std::snprintf(name + n, sizeof name - n, "%02x", id[i]);
    x.name = name;
    const int fd = ::shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) {
        std::snprintf(m->last_err, sizeof m->last_err, "shm_open %s: %s", name, std::strerror(errno));
        return RT_ERR_COMM;
    }
    void* p = MAP_FAILED;
    if (::ftruncate(fd, (off_t)sizeof(IpcShared)) == 0)
        p = ::mmap(nullptr, sizeof(IpcShared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    const int err = errno;
    ::close(fd);
    if (p == MAP_FAILED) {
        std::snprintf(m->last_err, sizeof m->last_err, "mapping %s: %s", name, std::strerror(err));
        return RT_ERR_COMM;
    }
    x.sh = static_cast<IpcShared*>(p);
    x.nrecv.assign((size_t)m->nranks, 0);
    x.nsent.assign((size_t)m->nranks, 0);
    Rank* k = m->r[0];
    DevGuard dg(k->device);
    MHIP(m, dg.err);
    IpcPeer& me = x.sh->peer[k->rank];
    if (ld_acq(&me.joined)) {
        std::snprintf(m->last_err, sizeof m->last_err, "IPC: rank %d joined %s twice", k->rank, name);
        return RT_ERR_INVALID_ARG;
    }
    me.pid = (int32_t)::getpid();
    me.nranks = m->nranks;
    st_rel(&me.joined, 1u);
    x.joined = true;
    int dead = -1;  // a rank that joined and whose process has exited since
    int st = ipc_wait(m, [&] {
        bool all = true;
        for (int g = 0; g < m->nranks; g++) {
            const IpcPeer& pg = x.sh->peer[g];
            if (!ld_acq(&pg.joined)) all = false;
            else if (g != k->rank && dead < 0 && pid_gone(pg.pid)) dead = g;
        }
        return all || dead >= 0;
    }, -1, "IPC: waiting for every rank to join", std::max<int64_t>(hub_timeout_ms(), 120000));
    if (st != RT_OK) return st;
    if (dead >= 0) {
        std::snprintf(m->last_err, sizeof m->last_err, "IPC: rank %d's process exited while the ranks joined", dead);
        return RT_ERR_COMM;
    }
    for (int g = 0; g < m->nranks; g++)
        if (x.sh->peer[g].nranks != m->nranks) {
            std::snprintf(m->last_err, sizeof m->last_err, "IPC: rank %d has %d ranks, this rank %d", g,
                          x.sh->peer[g].nranks, m->nranks);
            return RT_ERR_INVALID_ARG;
        }
    if (m->has_root()) {
        // every rank has the segment mapped: drop its name (nothing left in /dev/shm)
        ::shm_unlink(name);
        x.unlinked = true;
    }
    return RT_OK;
}
/* Before this rank's exported buffers are freed (and the segment unmapped): close what it
 * imported, mark it left, and wait (bounded) until every peer has done the same, so no peer
 * still uses them.  The streams were drained first, so no host function still runs. */
void ipc_leave(rt_multi* m) {
    if (!m->ipc) return;
    Ipc& x = *m->ipc;
    if (x.sh) {
        DevGuard dg(m->r.empty() ? 0 : m->r[0]->device);
        for (auto& o : x.opened) (void)hipIpcCloseMemHandle(o.second);
        x.opened.clear();
        if (x.joined && !m->r.empty()) {
            st_rel(&x.sh->peer[m->r[0]->rank].left, 1u);
            const auto t0 = std::chrono::steady_clock::now();
            for (int g = 0; g < m->nranks; g++) {
                IpcPeer& pg = x.sh->peer[g];
                while (ld_acq(&pg.joined) && !ld_acq(&pg.left) && !pid_gone(pg.pid) &&
                       std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(hub_timeout_ms()))
                    std::this_thread::sleep_for(std::chrono::microseconds(200));
            }
        }
        ::munmap(x.sh, sizeof(IpcShared));
        x.sh = nullptr;
    }
    if (!x.unlinked && !x.name.empty() && m->has_root()) ::shm_unlink(x.name.c_str());
    x.unlinked = true;
    // the root's exported staging buffers (the rank's pointers to them are dropped)
    if (!m->r.empty()) {
        Rank* k = m->r[0];
        for (auto& b : k->staging) b = nullptr;
        for (auto& b : k->bstage) b = nullptr;
    }
    for (auto& e : x.exp) (void)hipFree(e.base);
    x.exp.clear();
}

/* rt_multi_render_device_frames in batches of m->batch frames (RT_OPT_MULTI_BATCH; the
 * caller checked the arguments and that the batched exchange applies). */
int render_batches(rt_multi* m, const rt_camera* cams, int32_t ncams, int32_t depth, int32_t precision,
                   uint32_t flags, int32_t out_format, void* const* d_frames, int32_t nbufs,
                   void* const* streams, int32_t nstreams, int32_t nframes) {
    Rank* k = m->r[0];
    DevGuard dg(k->device);
    MHIP(m, dg.err);
    const bool root = m->has_root();
    std::vector<hipStream_t> uniq_all;
    int last_bs = 0;
    for (int32_t b0 = 0; b0 < nframes; b0 += m->batch) {
        const int kb = (int)std::min<int32_t>(m->batch, nframes - b0);
        rt_camera cb[RT_MULTI_BATCH_MAX];
        for (int i = 0; i < kb; i++) cb[i] = cams[(b0 + i) % ncams];
        BatchJob b;
        b.cams = cb;
        b.kb = kb;
        b.bs = (int)(m->nbatch % 2);
        b.depth = depth;
        b.precision = precision;
        b.flags = flags;
        b.out_format = out_format;
        m->queued.store(false, std::memory_order_relaxed);
        int st;
        if (root) {
            char* fr[RT_MULTI_BATCH_MAX];
            hipStream_t ss[RT_MULTI_BATCH_MAX];
            std::vector<hipStream_t> uniq;
            for (int i = 0; i < kb; i++) {
                const int32_t f = b0 + i;
                fr[i] = static_cast<char*>(d_frames[f % nbufs]);
                void* cs = nstreams > 0 ? streams[f % nstreams] : nullptr;
                ss[i] = cs ? static_cast<hipStream_t>(cs) : k->render_stream[f % m->slots];
                if (std::find(uniq.begin(), uniq.end(), ss[i]) == uniq.end()) uniq.push_back(ss[i]);
            }
            st = batch_root(m, k, b, fr, ss, uniq);
            for (hipStream_t u : uniq)
                if (std::find(uniq_all.begin(), uniq_all.end(), u) == uniq_all.end()) uniq_all.push_back(u);
        } else {
            st = batch_send(m, k, b, false);
        }
        m->frame += (uint64_t)kb;
        m->nbatch++;
        if (st != RT_OK) {
            mark_failed(m);
            return st;
        }
        last_bs = b.bs;
    }
    // the caller's streams see the complete frames (root) / follow the last send
    if (root) {
        for (hipStream_t u : uniq_all) MHIPF(m, hipStreamWaitEvent(u, k->ev_done, 0));
    } else {
        for (int32_t s = 0; s < nstreams && s < nframes; s++)
            if (streams[s]) MHIPF(m, hipStreamWaitEvent(static_cast<hipStream_t>(streams[s]), k->ev_bsent[last_bs], 0));
    }
    return RT_OK;
}

/* One frame of rt_multi_render_device (arguments already checked). */
int render_frame(rt_multi* m, const rt_camera* cam, int32_t depth, int32_t precision, uint32_t flags,
                 int32_t out_format, void* d_frame, void* stream) {
    if (m->broken) {
        std::snprintf(m->last_err, sizeof m->last_err,
                      "an earlier frame failed after the gather was queued: the communicator is out of step");
        return RT_ERR_COMM;
    }
    const int slot = (int)(m->frame % (uint64_t)m->slots);
    m->queued.store(false, std::memory_order_relaxed);
    Job j;
    j.cam = cam;
    j.depth = depth;
    j.precision = precision;
    j.flags = flags;
    j.out_format = out_format;
    j.d_frame = static_cast<char*>(d_frame);
    j.slot = slot;
    Rank* root = m->has_root() ? m->r[0] : nullptr;
    if (root) {
        if (!d_frame && (size_t)cam->width * cam->height > 0) return RT_ERR_INVALID_ARG;
        DevGuard dg(root->device);
        MHIP(m, dg.err);
        j.stream = stream ? static_cast<hipStream_t>(stream) : root->render_stream[slot];
        j.ev_in = m->ev_in[slot];
        // one rank: the band is the frame, rendered in place in stream order; nothing else
        // writes the frame buffer, so no event is needed (it costs host time every frame)
        if (m->nranks > 1 || m->gathers()) MHIPF(m, hipEventRecord(j.ev_in, j.stream));
    } else {
        j.stream = static_cast<hipStream_t>(stream);
    }
    // the extra local ranks on their worker threads, the first on this thread
    for (int L = 1; L < m->nlocal; L++) {
        Rank* k = m->r[L];
        {
            std::lock_guard<std::mutex> lk(k->mu);
            k->job = j;
            k->job.stream = nullptr;  // only the process's first rank sees the caller's stream
            k->posted.store(m->frame + 1, std::memory_order_release);
        }
        k->cv.notify_one();
    }
    int st = enqueue_rank(m, m->r[0], j);
    {
        SlowCall sc_("waiting for the worker threads");
        for (int L = 1; L < m->nlocal; L++) {
            Rank* k = m->r[L];
            while (k->finished.load(std::memory_order_acquire) != m->frame + 1) std::this_thread::yield();
            if (st == RT_OK && k->status != RT_OK) st = k->status;
        }
    }
    m->frame++;
    if (st != RT_OK) {
        mark_failed(m);
        return st;
    }
    if (root && (m->nranks > 1 || m->gathers())) {
        // the caller's stream sees the complete frame
        DevGuard dg(root->device);
        MHIP(m, dg.err);
        if (m->rccl() || m->threads()) {
            MHIPF(m, hipStreamWaitEvent(j.stream, root->ev_done, 0));
        } else {
            for (int L = 1; L < m->nlocal; L++) MHIPF(m, hipStreamWaitEvent(j.stream, m->r[L]->ev_sent[slot], 0));
        }
    }
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_multi_unique_id(uint8_t id[RT_MULTI_ID_BYTES]) {
    if (!id) return RT_ERR_INVALID_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return RT_ERR_COMM;
    static_assert(sizeof u == RT_MULTI_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof u);
    return RT_OK;
}

const char* rt_multi_last_error(const rt_multi* m) { return m ? m->last_err : ""; }

int rt_multi_create(const int32_t* devices, int32_t nlocal, int32_t nranks, int32_t first_rank,
                    const uint8_t* unique_id, int32_t transport, rt_multi** out) {
    if (!out) return RT_ERR_INVALID_ARG;
    *out = nullptr;
    if (!devices || nlocal <= 0 || nranks <= 0 || first_rank < 0 || first_rank + nlocal > nranks)
        return RT_ERR_INVALID_ARG;
    if (transport != RT_TRANSPORT_RCCL && transport != RT_TRANSPORT_COPY &&
        transport != RT_TRANSPORT_RCCL_LOOPBACK && transport != RT_TRANSPORT_THREADS &&
        transport != RT_TRANSPORT_IPC)
        return RT_ERR_INVALID_ARG;
    const bool one_process = nlocal == nranks;
    if (!one_process && (!unique_id || transport == RT_TRANSPORT_COPY))
        return transport == RT_TRANSPORT_COPY ? RT_ERR_UNSUPPORTED : RT_ERR_INVALID_ARG;
    // THREADS / IPC: one handle per rank (the process-per-GPU shape), two ranks at least
    if ((transport == RT_TRANSPORT_THREADS || transport == RT_TRANSPORT_IPC) && (nlocal != 1 || nranks < 2))
        return RT_ERR_INVALID_ARG;
    if (transport == RT_TRANSPORT_IPC && (!unique_id || nranks > IPC_MAX_RANKS)) return RT_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_ERR_NO_DEVICE;
    for (int L = 0; L < nlocal; L++)
        if (devices[L] < 0 || devices[L] >= ndev) return RT_ERR_NO_DEVICE;
    if (transport != RT_TRANSPORT_COPY && transport != RT_TRANSPORT_THREADS && transport != RT_TRANSPORT_IPC)
        for (int a = 0; a < nlocal; a++)
            for (int b = a + 1; b < nlocal; b++)
                if (devices[a] == devices[b]) return RT_ERR_UNSUPPORTED;  // RCCL: one rank per GPU

    rt_multi* m = new (std::nothrow) rt_multi();
    if (!m) return RT_ERR_OUT_OF_MEMORY;
    m->nranks = nranks;
    m->nlocal = nlocal;
    m->first_rank = first_rank;
    m->transport = transport;
    int st = RT_OK;
    auto fail = [&](int s) {
        st = s;
        return s;
    };
    for (int L = 0; L < nlocal && st == RT_OK; L++) {
        Rank* k = new (std::nothrow) Rank();
        if (!k) {
            fail(RT_ERR_OUT_OF_MEMORY);
            break;
        }
        m->r.push_back(k);
        k->rank = first_rank + L;
        k->device = devices[L];
        int cs = rt_ctx_create(k->device, &k->ctx);
        if (cs != RT_OK) {
            fail(cs);
            break;
        }
        DevGuard dg(k->device);
        hipError_t e = dg.err;
        const unsigned xf = hipEventDisableTiming;
        for (auto& rs : k->render_stream)
            if (e == hipSuccess) e = hipStreamCreateWithFlags(&rs, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&k->comm_stream, hipStreamNonBlocking);
        for (int s = 0; s < RT_MULTI_SLOTS && e == hipSuccess; s++) {
            e = hipEventCreateWithFlags(&k->ev_rendered[s], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&k->ev_sent[s], xf);
            // recorded once, so the first wait on a slot (no send yet) is already satisfied
            if (e == hipSuccess) e = hipEventRecord(k->ev_sent[s], k->comm_stream);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&k->ev_ready[s], xf);
        }
        if (e == hipSuccess) e = hipEventCreateWithFlags(&k->ev_done, hipEventDisableTiming);
        for (int b = 0; b < 2 && e == hipSuccess; b++) {
            for (int j = 0; j < RT_MULTI_SLOTS && e == hipSuccess; j++)
                e = hipEventCreateWithFlags(&k->ev_brend[b][j], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&k->ev_bsent[b], xf);
            if (e == hipSuccess) e = hipEventRecord(k->ev_bsent[b], k->comm_stream);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&k->ev_bdone[b], hipEventDisableTiming);
        }
        for (auto& ev : k->ev_drain)
            if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        for (auto& ev : k->ev_rows)
            if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) fail(hip_err(m, e, "rank streams/events"));
    }
    if (st == RT_OK && m->has_root()) {
        DevGuard dg(m->r[0]->device);
        hipError_t e = dg.err;
        for (int s = 0; s < RT_MULTI_SLOTS && e == hipSuccess; s++)
            e = hipEventCreateWithFlags(&m->ev_in[s], hipEventDisableTiming);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&m->host_stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreate(&m->ev0);
        if (e == hipSuccess) e = hipEventCreate(&m->ev1);
        if (e != hipSuccess) fail(hip_err(m, e, "root streams/events"));
        if (st == RT_OK && transport == RT_TRANSPORT_COPY) {
            // direct xGMI peer copies where the devices allow it (else the runtime stages)
            for (int L = 1; L < nlocal; L++) {
                const int d = m->r[L]->device, d0 = m->r[0]->device;
                int can = 0;
                if (d != d0 && hipDeviceCanAccessPeer(&can, d, d0) == hipSuccess && can) {
                    DevGuard g2(d);
                    const hipError_t pe = hipDeviceEnablePeerAccess(d0, 0);
                    if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled)
                        (void)hipGetLastError();
                    else if (pe == hipErrorPeerAccessAlreadyEnabled)
                        (void)hipGetLastError();
                }
            }
        }
    }
    if (st == RT_OK && m->threads()) {
        // the mailbox of this unique id, shared with the other ranks' handles
        m->hub_key.assign(reinterpret_cast<const char*>(unique_id), RT_MULTI_ID_BYTES);
        std::lock_guard<std::mutex> lk(g_hubs_mu);
        auto& h = g_hubs[m->hub_key];
        if (!h) h = std::make_shared<Hub>();
        m->hub = h;
        std::lock_guard<std::mutex> lk2(h->mu);
        h->refs++;
    }
    if (st == RT_OK && transport == RT_TRANSPORT_IPC) fail(ipc_create(m, unique_id));
    // one rank: the band is the frame and nothing is exchanged, so no communicator (RCCL's
    // init would only print its banner on stdout and start its proxy thread) — except for
    // the loopback transport, whose root sends its band to itself
    if (st == RT_OK && m->gathers() && m->rccl()) {
        ncclUniqueId id;
        if (one_process && !unique_id) {
            if (ncclGetUniqueId(&id) != ncclSuccess) fail(nccl_err(m, ncclInternalError, "ncclGetUniqueId"));
        } else {
            std::memcpy(&id, unique_id, sizeof id);
        }
        if (st == RT_OK) {
            // one rank per device; several local ranks join inside one group (what
            // ncclCommInitAll does)
            ncclResult_t e = nlocal > 1 ? ncclGroupStart() : ncclSuccess;
            for (int L = 0; L < nlocal && e == ncclSuccess; L++) {
                DevGuard dg(m->r[L]->device);
                e = ncclCommInitRank(&m->r[L]->comm, nranks, id, m->r[L]->rank);
            }
            const ncclResult_t e2 = nlocal > 1 ? ncclGroupEnd() : ncclSuccess;
            if (e != ncclSuccess || e2 != ncclSuccess)
                fail(nccl_err(m, e != ncclSuccess ? e : e2, "ncclCommInitRank"));
        }
    }
    if (st == RT_OK) {
        for (int L = 1; L < nlocal; L++) {
            Rank* k = m->r[L];
            try {
                k->th = std::thread(worker_main, m, k);
            } catch (...) {
                fail(RT_ERR_OUT_OF_MEMORY);
                break;
            }
        }
    }
    if (st != RT_OK) {
        std::fprintf(stderr, "rt_multi_create: %s %s\n", rt_strerror(st), m->last_err);
        rt_multi_destroy(m);
        return st;
    }
    *out = m;
    return RT_OK;
}

/* A broken rt_multi: abort every local communicator once (pending receives that can no
 * longer complete are cancelled, so the streams can drain). */
void abort_comms(rt_multi* m) {
    if (m->aborted) return;
    m->aborted = true;
    for (Rank* k : m->r)
        if (k->comm) {
            DevGuard dg(k->device);
            (void)ncclCommAbort(k->comm);
            k->comm = nullptr;
        }
}

/* Waits for every local rank's streams by polling (a blocking wait could never end when a
 * peer process died with its part of the exchange outstanding): an event recorded at the end
 * of each stream is polled (hipStreamQuery was seen to report a stream done while its last
 * command, a cross-stream wait, was still pending), RCCL's asynchronous error is checked
 * while waiting, and when it reports one or timeout_ms (> 0) passes, the exchange is broken,
 * the communicators are aborted and RT_ERR_COMM is returned. */
static int drain_streams(rt_multi* m, int64_t timeout_ms) {
    const auto t0 = std::chrono::steady_clock::now();
    for (Rank* k : m->r) {
        DevGuard dg(k->device);
        MHIP(m, dg.err);
        hipStream_t ss[RT_MULTI_SLOTS + 1];
        for (int s = 0; s < RT_MULTI_SLOTS; s++) ss[s] = k->render_stream[s];
        ss[RT_MULTI_SLOTS] = k->comm_stream;
        for (int i = 0; i <= RT_MULTI_SLOTS; i++)
            if (ss[i]) MHIP(m, hipEventRecord(k->ev_drain[i], ss[i]));
        for (int i = 0; i <= RT_MULTI_SLOTS; i++) {
            if (!ss[i]) continue;
            for (int it = 0;; it++) {
                const hipError_t e = hipEventQuery(k->ev_drain[i]);
                if (e == hipSuccess) break;
                if (e != hipErrorNotReady) return hip_err(m, e, "hipEventQuery");
                const char* why = nullptr;
                ncclResult_t async = ncclSuccess;
                if (k->comm && (it & 63) == 0 && (ncclCommGetAsyncError(k->comm, &async) != ncclSuccess ||
                                                  async != ncclSuccess))
                    why = async != ncclSuccess ? ncclGetErrorString(async) : "ncclCommGetAsyncError failed";
                else if (timeout_ms > 0 && (it & 15) == 0 &&
                         std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms))
                    why = "deadline passed (RT_OPT_MULTI_TIMEOUT_MS)";
                if (why) {
                    std::snprintf(m->last_err, sizeof m->last_err,
                                  "rt_multi_sync (rank %d): %s with its exchange outstanding: communicator aborted",
                                  k->rank, why);
                    if (!m->broken) {
                        m->broken = true;
                        hub_fail(m);
                        ipc_fail(m);
                    }
                    abort_comms(m);
                    return RT_ERR_COMM;
                }
                if (it < 1024) std::this_thread::yield();
                else std::this_thread::sleep_for(std::chrono::microseconds(50));
            }
        }
        if (k->comm) {
            ncclResult_t async = ncclSuccess;
            MNCCL(m, ncclCommGetAsyncError(k->comm, &async));
            if (async != ncclSuccess) {
                m->broken = true;
                abort_comms(m);
                return nccl_err(m, async, "ncclCommGetAsyncError");
            }
        }
    }
    return RT_OK;
}

int rt_multi_destroy(rt_multi* m) {
    if (!m) return RT_ERR_INVALID_ARG;
    if (m->broken) abort_comms(m);
    // THREADS: peers still waiting on this handle give up, and its posts (naming its events)
    // are withdrawn before the events are destroyed
    if (m->hub) hub_leave(m);
    if (m->ipc) {
        // IPC: this rank's streams drained, its imports closed, and the peers' likewise
        // before its exported events and staging buffers go (ipc_leave waits for them)
        for (Rank* k : m->r) {
            DevGuard dg(k->device);
            for (auto rs : k->render_stream)
                if (rs) (void)hipStreamSynchronize(rs);
            if (k->comm_stream) (void)hipStreamSynchronize(k->comm_stream);
        }
        ipc_leave(m);
    }
    for (Rank* k : m->r) destroy_rank(k, m->broken);
    m->r.clear();
    m->ipc.reset();
    if (m->hub) {
        // the last handle drops the mailbox
        std::lock_guard<std::mutex> lk(g_hubs_mu);
        bool last;
        {
            std::lock_guard<std::mutex> lk2(m->hub->mu);
            last = --m->hub->refs == 0;
        }
        if (last) g_hubs.erase(m->hub_key);
        m->hub.reset();
    }
    // the root's device objects (every rank has been synchronised above)
    for (auto& e : m->ev_in)
        if (e) (void)hipEventDestroy(e);
    if (m->ev0) (void)hipEventDestroy(m->ev0);
    if (m->ev1) (void)hipEventDestroy(m->ev1);
    if (m->host_stream) (void)hipStreamDestroy(m->host_stream);
    if (m->d_frame) (void)hipFree(m->d_frame);
    delete m;
    return RT_OK;
}

int rt_multi_set_scene(rt_multi* m, const rt_prim* prims, int32_t n) {
    if (!m) return RT_ERR_INVALID_ARG;
    for (Rank* k : m->r) {
        const int st = rt_set_scene(k->ctx, prims, n);
        if (st != RT_OK) return ctx_err(m, k, st, "rt_set_scene");
    }
    return RT_OK;
}

int rt_multi_set_option(rt_multi* m, int32_t option, int64_t value) {
    if (!m) return RT_ERR_INVALID_ARG;
    if (option == RT_OPT_MULTI_FAULT) {
        if (value != 0 && value != 1) return RT_ERR_INVALID_ARG;
        m->fault_next = value == 1;
        return RT_OK;
    }
    if (option == RT_OPT_MULTI_FRAMES) {
        if (value < 1 || value > RT_MULTI_SLOTS) return RT_ERR_INVALID_ARG;
        const int st = rt_multi_sync(m);  // frames in flight keep the slots they started with
        if (st != RT_OK) return st;
        m->slots = (int)value;
        return RT_OK;
    }
    if (option == RT_OPT_MULTI_TIMEOUT_MS) {
        if (value < 0) return RT_ERR_INVALID_ARG;
        m->timeout_ms = value;
        return RT_OK;
    }
    if (option == RT_OPT_MULTI_BATCH) {
        if (value < 1 || value > RT_MULTI_BATCH_MAX) return RT_ERR_INVALID_ARG;
        m->batch = (int)value;  // takes effect from the next rt_multi_render_device_frames
        return RT_OK;
    }
    if (option == RT_OPT_FRAME_BATCH) {
        if (value < 1 || value > RT_MULTI_BATCH_MAX) return RT_ERR_INVALID_ARG;
        for (Rank* k : m->r) {
            const int st = rt_set_option(k->ctx, option, value);
            if (st != RT_OK) return ctx_err(m, k, st, "rt_set_option");
        }
        m->frame_batch = (int)value;  // the batched exchange renders a batch on one stream
        return RT_OK;
    }
    if (option == RT_OPT_MULTI_LAYOUT) {
        if (value < 0 || value > 2) return RT_ERR_INVALID_ARG;
        const int st = rt_multi_sync(m);  // frames in flight keep the layout they started with
        if (st != RT_OK) return st;
        m->layout = (int)value;
        return RT_OK;
    }
    for (Rank* k : m->r) {
        const int st = rt_set_option(k->ctx, option, value);
        if (st != RT_OK) return ctx_err(m, k, st, "rt_set_option");
    }
    return RT_OK;
}

int rt_multi_set_row_weights(rt_multi* m, const float* weights, int32_t n) {
    if (!m || n < 0 || (n > 0 && !weights)) return RT_ERR_INVALID_ARG;
    for (int32_t t = 0; t < n; t++)
        if (!valid_weight(weights[t])) return RT_ERR_INVALID_ARG;
    const int st = rt_multi_sync(m);  // frames in flight keep the bands they started with
    if (st != RT_OK) return st;
    m->weights.assign(weights, weights + n);
    return RT_OK;
}

int rt_weighted_band_rows(int32_t height, int32_t nranks, int32_t rank, const float* weights,
                          int32_t n, int32_t* row0, int32_t* nrows) {
    if (!row0 || !nrows || height < 0 || nranks <= 0 || rank < 0 || rank >= nranks || n < 0)
        return RT_ERR_INVALID_ARG;
    const int32_t TH = rt_tile_rows(), T = (height + TH - 1) / TH;
    if (n != T || (n > 0 && !weights)) return RT_ERR_INVALID_ARG;
    // prefix sums in double, in a fixed order: every rank computes the same boundaries
    std::vector<double> P((size_t)T + 1, 0.0);
    for (int32_t t = 0; t < T; t++) {
        if (!valid_weight(weights[t])) return RT_ERR_INVALID_ARG;
        P[t + 1] = P[t] + (double)weights[t];
    }
    const double total = P[T];
    auto boundary = [&](int32_t r) -> int32_t {  // tile row where band r starts
        if (r <= 0) return 0;
        if (r >= nranks) return T;
        if (!(total > 0.0)) return (int32_t)(((int64_t)T * r) / nranks);  // no weight: equal tile rows
        const double target = total * r / nranks;
        // first t with P[t] >= target, then the nearer of t - 1 and t (ties: the lower)
        int32_t t = (int32_t)(std::lower_bound(P.begin(), P.end(), target) - P.begin());
        if (t > T) t = T;
        if (t > 0 && target - P[t - 1] <= P[t] - target) t--;
        return t;
    };
    int32_t b0 = 0, b1 = 0;
    for (int32_t r = 1; r <= rank + 1; r++) {  // non-decreasing boundaries
        const int32_t b = std::max(b1, boundary(r));
        b0 = b1;
        b1 = b;
    }
    *row0 = std::min(height, b0 * TH);
    *nrows = std::min(height, b1 * TH) - *row0;
    return RT_OK;
}

int rt_multi_render_device(rt_multi* m, const rt_camera* cam, int32_t depth, int32_t precision,
                           uint32_t flags, int32_t out_format, void* d_frame, void* stream) {
    const int st = check_args(m, cam, depth, precision, out_format);
    if (st != RT_OK) return st;
    return render_frame(m, cam, depth, precision, flags, out_format, d_frame, stream);
}

int rt_multi_render_device_frames(rt_multi* m, const rt_camera* cams, int32_t ncams,
                                  int32_t depth, int32_t precision, uint32_t flags,
                                  int32_t out_format, void* const* d_frames, int32_t nbufs,
                                  void* const* streams, int32_t nstreams, int32_t nframes) {
    if (!m || !cams || ncams <= 0 || nframes < 0 || nbufs < 0 || nstreams < 0 ||
        (nbufs > 0 && !d_frames) || (nstreams > 0 && !streams))
        return RT_ERR_INVALID_ARG;
    if (m->has_root() && nbufs == 0) return RT_ERR_INVALID_ARG;
    if (m->nranks == 1 && !m->gathers() && !m->broken && nstreams > 0 && nframes > 1) {
        // one rank and no exchange: the band is the frame, rendered in place on the caller's
        // streams, so the batch is the ctx's own frame loop (rt_render_device_frames, with
        // its host pipeline) — the same launches as frame-by-frame render_frame
        bool same = true;
        for (int32_t s = 0; s < nstreams; s++) same = same && streams[s] != nullptr;
        for (int32_t c = 0; c < ncams && c < nframes; c++)
            same = same && cams[c].height == cams[0].height &&
                   check_args(m, &cams[c], depth, precision, out_format) == RT_OK;
        if (same) {
            Rank* k = m->r[0];
            const int st = ctx_err(m, k,
                                   rt_render_device_frames(k->ctx, cams, ncams, 0, cams[0].height, depth,
                                                           precision, flags, out_format, d_frames, nbufs,
                                                           streams, nstreams, nframes),
                                   "rt_render_device_frames");
            m->frame += (uint64_t)nframes;
            return st;
        }
    }
    if (m->batch > 1 && nframes >= 2 && m->nlocal == 1 && m->gathers() && !m->broken &&
        !(m->layout == 1 && m->nranks > 1)) {
        // the batched exchange.  Whether a call batches must be the same on every rank (the
        // root's receives match the senders' sends), so it depends only on what every rank
        // is given alike: the option, the frame count, the cameras (every frame the same
        // size, so the bands are fixed, and valid).  What only the root is given must then
        // fit: at most RT_MULTI_SLOTS caller streams (one ev_in each), non-NULL buffers, and
        // a distinct buffer for every frame of a batch (frames of one batch sharing a buffer
        // could never be whole in it: the later frame's rows would land before the earlier
        // frame's other rows).  A refusal is returned before anything is enqueued here; with
        // ranks in other processes their sends of this call are then unmatched, so the
        // exchange is broken (mark_failed; the mailbox transports tell the peers).
        bool ok = true;
        for (int32_t c = 0; c < ncams && c < nframes && ok; c++)
            ok = cams[c].width == cams[0].width && cams[c].height == cams[0].height &&
                 check_args(m, &cams[c], depth, precision, out_format) == RT_OK;
        if (ok && m->has_root()) {
            std::vector<void*> uniq;  // as render_batches picks them
            for (int32_t f = 0; f < nframes && uniq.size() <= (size_t)RT_MULTI_SLOTS; f++) {
                void* cs = nstreams > 0 ? streams[f % nstreams] : nullptr;
                if (!cs) cs = m->r[0]->render_stream[f % m->slots];
                if (std::find(uniq.begin(), uniq.end(), cs) == uniq.end()) uniq.push_back(cs);
            }
            bool bufs = true;
            for (int32_t f = 0; f < nframes && f < nbufs && bufs; f++)
                bufs = d_frames[f] != nullptr || (size_t)cams[0].width * cams[0].height == 0;
            const int32_t kb0 = std::min<int32_t>(m->batch, nframes);
            std::vector<void*> dist;
            for (int32_t f = 0; f < kb0; f++)
                if (std::find(dist.begin(), dist.end(), d_frames[f % nbufs]) == dist.end())
                    dist.push_back(d_frames[f % nbufs]);
            const bool whole = (int32_t)dist.size() >= kb0 || (size_t)cams[0].width * cams[0].height == 0;
            if (uniq.size() > (size_t)RT_MULTI_SLOTS || !bufs || !whole) {
                if (!whole)
                    std::snprintf(m->last_err, sizeof m->last_err,
                                  "RT_OPT_MULTI_BATCH %d: %d distinct frame buffers for a batch of %d frames "
                                  "(each frame of a batch needs its own buffer)", m->batch, (int)dist.size(), kb0);
                else
                    std::snprintf(m->last_err, sizeof m->last_err,
                                  "RT_OPT_MULTI_BATCH: the root takes at most %d distinct caller streams and "
                                  "non-NULL frame buffers", RT_MULTI_SLOTS);
                if (m->nlocal < m->nranks) mark_failed(m);
                return bufs ? RT_ERR_UNSUPPORTED : RT_ERR_INVALID_ARG;
            }
        }
        if (ok)
            return render_batches(m, cams, ncams, depth, precision, flags, out_format, d_frames, nbufs,
                                  streams, nstreams, nframes);
    }
    for (int32_t f = 0; f < nframes; f++) {
        const rt_camera* cam = &cams[f % ncams];
        int st = check_args(m, cam, depth, precision, out_format);
        if (st != RT_OK) return st;
        st = render_frame(m, cam, depth, precision, flags, out_format,
                          nbufs > 0 ? d_frames[f % nbufs] : nullptr,
                          nstreams > 0 ? streams[f % nstreams] : nullptr);
        if (st != RT_OK) return st;
    }
    return RT_OK;
}

int rt_multi_render(rt_multi* m, const rt_camera* cam, int32_t depth, int32_t precision,
                    uint32_t flags, int32_t out_format, void* out, rt_stats* stats) {
    int st = check_args(m, cam, depth, precision, out_format);
    if (st != RT_OK) return st;
    const size_t bytes = (size_t)cam->width * cam->height * bpp(out_format);
    if (!m->has_root()) {
        st = render_frame(m, cam, depth, precision, flags, out_format, nullptr, nullptr);
        if (st != RT_OK) return st;
        if (stats) *stats = rt_stats{0.0, 0};
        return rt_multi_sync(m);
    }
    if (!out && bytes > 0) return RT_ERR_INVALID_ARG;
    Rank* root = m->r[0];
    {
        DevGuard dg(root->device);
        MHIP(m, dg.err);
        if (bytes > m->d_frame_cap) {
            MHIP(m, hipStreamSynchronize(m->host_stream));
            if (m->d_frame) MHIP(m, hipFree(m->d_frame));
            m->d_frame = nullptr;
            m->d_frame_cap = 0;
            MHIP(m, hipMalloc(&m->d_frame, bytes));
            m->d_frame_cap = bytes;
        }
        MHIP(m, hipEventRecord(m->ev0, m->host_stream));
    }
    st = render_frame(m, cam, depth, precision, flags, out_format, m->d_frame, m->host_stream);
    if (st != RT_OK) return st;
    DevGuard dg(root->device);
    MHIP(m, dg.err);
    MHIP(m, hipEventRecord(m->ev1, m->host_stream));
    if (bytes > 0) MHIP(m, hipMemcpyAsync(out, m->d_frame, bytes, hipMemcpyDeviceToHost, m->host_stream));
    MHIP(m, hipStreamSynchronize(m->host_stream));
    st = rt_multi_sync(m);
    if (st != RT_OK) return st;
    if (stats) {
        float ms = 0.f;
        MHIP(m, hipEventElapsedTime(&ms, m->ev0, m->ev1));
        stats->ms = ms;
        stats->segments = 0;
    }
    return RT_OK;
}

int rt_multi_sync(rt_multi* m) {
    if (!m) return RT_ERR_INVALID_ARG;
    if (m->broken) {
        abort_comms(m);
        (void)drain_streams(m, 10000);
        std::snprintf(m->last_err, sizeof m->last_err, "a frame failed after the gather was queued: communicator aborted");
        return RT_ERR_COMM;
    }
    return drain_streams(m, m->timeout_ms);
}

}  // extern "C"
