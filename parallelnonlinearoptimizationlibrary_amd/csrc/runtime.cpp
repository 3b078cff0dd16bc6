// runtime.cpp -- contexts, device memory, workspace and the communicator behind the C ABI.
//
// The communicator replaces MPI_COMM_WORLD on the paths the reference distributes
// (PNOL_Objective.cpp:101-103, 147-148, 226-228, 279-288; BFGS_with_linesearch_MPI.cpp:167-210):
// RCCL (one process per GPU, xGMI) or a caller-supplied host allgather (tests / host objectives).
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>

#include "pnol_comm.hpp"

#include <algorithm>
#include "pnol_internal.hpp"

namespace pnol {

int ws_get(pnol_ctx* ctx, const char* key, size_t bytes, void** out, bool* fresh) {
    if (!ctx || !out) return PNOL_ERR_ARG;
    auto& slot = ctx->ws.bufs[key];
    if (fresh) *fresh = false;
    if (slot.second < bytes) {
        if (fresh) *fresh = true;   // new contents, even when the allocator hands back the old address
        if (slot.first) {
            PNOL_CHECK(stream_wait(ctx->stream));
            PNOL_HIP(hipFree(slot.first));
            slot.first = nullptr;
            slot.second = 0;
        }
        size_t sz = bytes < 256 ? 256 : bytes;
        if (hipMalloc(&slot.first, sz) != hipSuccess) {
            slot.first = nullptr;
            return PNOL_ERR_NOMEM;
        }
        slot.second = sz;
    }
    *out = slot.first;
    return PNOL_OK;
}

// ws_get whose buffer reads as zero when (re)allocated (flag / counter arrays)
int ws_get_zeroed(pnol_ctx* ctx, const char* key, size_t bytes, void** out) {
    if (!ctx || !out) return PNOL_ERR_ARG;
    bool fresh = false;
    PNOL_CHECK(ws_get(ctx, key, bytes, out, &fresh));
    if (fresh) PNOL_HIP(hipMemsetAsync(*out, 0, ctx->ws.bufs[key].second, ctx->stream));
    return PNOL_OK;
}

static bool is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

// ---------------------------------------------------------------------------------------
// communicator
// ---------------------------------------------------------------------------------------
struct CommState {
    int kind = 0;   // 0 none (single process), 1 rccl, 2 host callback
    int nranks = 1, rank = 0;
    ncclComm_t nccl = nullptr;
    bool dead = false;   // aborted after a stuck or failed exchange: every later collective fails
    pnol_ctx* ctx = nullptr;
    pnol_host_allgather_fn fn = nullptr;
    void* user = nullptr;
};
static CommState g_comm;

int comm_size() { return g_comm.nranks; }
int comm_rank() { return g_comm.rank; }

// MPI launcher binding: the hook is compiled into the user's program against its own MPI
// (include/pnol_mpi_bind.hpp); the library only calls it.
static pnol_launcher_hook_fn g_launch_hook = nullptr;
static bool g_launch_bound = false;
static std::mutex g_launch_mu;

static int env_int(const char* name, int dflt) {
    const char* e = std::getenv(name);
    if (!e || !*e) return dflt;
    char* end = nullptr;
    const long v = std::strtol(e, &end, 10);
    return (end && *end == 0) ? (int)v : dflt;
}

int launcher_world_size() {
    for (const char* k : {"PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "MV2_COMM_WORLD_SIZE"}) {
        const int v = env_int(k, 0);
        if (v > 0) return v;
    }
    return 1;
}

int comm_bind_launcher() {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    if (g_comm.kind != 0) return PNOL_OK;
    if (g_launch_hook && !g_launch_bound) {
        const int st = g_launch_hook();
        if (st == 0) g_launch_bound = true;
        if (st < 0) {
            std::fprintf(stderr, "pnol_amd: the MPI launcher binding failed (status %d)\n", st);
            return PNOL_ERR_COMM;
        }
    }
    const int ws = launcher_world_size();
    if (g_comm.kind == 0 && ws > 1) {
        std::fprintf(stderr,
                     "pnol_amd: this process was started by an MPI launcher with %d ranks, but no communicator is "
                     "bound.  Call MPI_Init before the first *_MPI call and compile with <mpi.h> on the include "
                     "path (the drop-in headers then bind MPI_COMM_WORLD), or bootstrap one with "
                     "pnol_comm_init_rccl / pnol_comm_init_host.  A *_MPI class does not run a %d-rank job as one "
                     "rank.\n",
                     ws, ws);
        return PNOL_ERR_COMM;
    }
    return PNOL_OK;
}

// Bounded host waits.  With an RCCL communicator bound, a stuck exchange (a peer that died or
// never posted its side) would hang the blocking HIP wait forever: every host wait of the
// library then polls the stream / event, checks ncclCommGetAsyncError every millisecond, and
// past PNOL_COMM_TIMEOUT_S seconds (default 300) aborts the communicator (ncclCommAbort) and
// returns PNOL_ERR_COMM, so the job fails with an error instead of hanging.  Without RCCL the
// waits are the plain HIP ones.
static double comm_timeout_s() {   // read per wait (cheap beside a wait; tests change it)
    const char* e = std::getenv("PNOL_COMM_TIMEOUT_S");
    const double v = e ? std::atof(e) : 0.0;
    return v > 0.0 ? v : 300.0;
}

static int comm_abort(const char* why) {
    std::fprintf(stderr, "[pnol_amd] rank %d of %d: %s; aborting the RCCL communicator\n", g_comm.rank, g_comm.nranks,
                 why);
    if (g_comm.nccl) (void)ncclCommAbort(g_comm.nccl);
    g_comm.nccl = nullptr;
    g_comm.dead = true;
    return PNOL_ERR_COMM;
}

template <class Q>
static int bounded_poll(Q query) {
    const double limit = comm_timeout_s();
    const auto t0 = std::chrono::steady_clock::now();
    auto last = t0;
    for (;;) {
        const hipError_t q = query();
        if (q == hipSuccess) return PNOL_OK;
        if (q != hipErrorNotReady) return PNOL_ERR_HIP;
        const auto now = std::chrono::steady_clock::now();
        if (now - last >= std::chrono::milliseconds(1)) {
            last = now;
            ncclResult_t ae = ncclSuccess;
            if (g_comm.nccl && ncclCommGetAsyncError(g_comm.nccl, &ae) == ncclSuccess && ae != ncclSuccess &&
                ae != ncclInProgress)
                return comm_abort(ncclGetErrorString(ae));
            if (std::chrono::duration<double>(now - t0).count() > limit)
                return comm_abort("a device wait with RCCL operations in flight passed PNOL_COMM_TIMEOUT_S");
        }
    }
}

int stream_wait(hipStream_t st) {
    if (g_comm.kind != 1 || !g_comm.nccl) return hipStreamSynchronize(st) == hipSuccess ? PNOL_OK : PNOL_ERR_HIP;
    return bounded_poll([st] { return hipStreamQuery(st); });
}

int event_wait(hipEvent_t ev) {
    if (g_comm.kind != 1 || !g_comm.nccl) {
        for (;;) {   // busy-poll (a blocking wait returns tens of microseconds late)
            const hipError_t q = hipEventQuery(ev);
            if (q == hipSuccess) return PNOL_OK;
            if (q != hipErrorNotReady) return PNOL_ERR_HIP;
        }
    }
    return bounded_poll([ev] { return hipEventQuery(ev); });
}

bool comm_dead() { return g_comm.kind == 1 && g_comm.dead; }

// several ranks over the host backend: the tests' and a one-GPU MPI launch's ranks share a GPU
bool comm_shares_device() { return g_comm.kind == 2 && g_comm.nranks > 1; }

void block_range(int ncols, int nranks, int rank, int* begin, int* count) {
    // ceil-sized contiguous blocks: the padded allgather buffer is then the row-major JT itself
    int per = (ncols + nranks - 1) / nranks;
    int b = rank * per;
    if (b > ncols) b = ncols;
    int e = b + per;
    if (e > ncols) e = ncols;
    *begin = b;
    *count = e - b;
}

// Cost-balanced FD column tiles: the ceil(ncols / tile) tiles are dealt to the ranks in
// snake order (0, 1, .., P-1, P-1, .., 0, 0, 1, ..).  With prefix sharing the cost of FD
// column j falls linearly with j, so each rank's sum pairs an expensive tile with a cheap
// one; contiguous blocks would leave rank 0 with ~2x the mean work at P = 8.
int fd_tile_owner(int tile, int nranks) {
    const int round = tile / nranks, pos = tile % nranks;
    return (round & 1) ? nranks - 1 - pos : pos;
}

void fd_tiles_of(int ncols, int nranks, int rank, std::vector<int>& start, std::vector<int>& count) {
    start.clear();
    count.clear();
    const int nt = (ncols + kFdTileCols - 1) / kFdTileCols;
    for (int t = 0; t < nt; ++t) {
        if (fd_tile_owner(t, nranks) != rank) continue;
        start.push_back(t * kFdTileCols);
        count.push_back(std::min(kFdTileCols, ncols - t * kFdTileCols));
    }
}

// Every rank ends with all ncols rows of buf (row c at buf + c * ld); rank r contributes the
// rows of its fd_tiles_of tiles.  RCCL: one group of point-to-point sends / receives straight
// into place (each tile goes owner -> every peer over its own xGMI link).  Host backend:
// pack, allgather through host memory, unpack.
int comm_share_rows(pnol_ctx* ctx, double* buf, size_t ld, int ncols) {
    const int P = g_comm.nranks, me = g_comm.rank;
    if (g_comm.kind == 0 || P == 1) return PNOL_OK;
    const int nt = (ncols + kFdTileCols - 1) / kFdTileCols;
    if (g_comm.kind == 1) {
        if (!g_comm.nccl) return PNOL_ERR_COMM;
        ScopedTimer tm(ctx, "allgather");
        if (ncclGroupStart() != ncclSuccess) return PNOL_ERR_COMM;
        for (int t = 0; t < nt; ++t) {
            const int o = fd_tile_owner(t, P);
            const size_t c0 = (size_t)t * kFdTileCols, rows = std::min(kFdTileCols, ncols - t * kFdTileCols);
            double* p = buf + c0 * ld;
            if (o == me) {
                for (int q = 0; q < P; ++q)
                    if (q != me && ncclSend(p, rows * ld, ncclDouble, q, g_comm.nccl, ctx->stream) != ncclSuccess) {
                        ncclGroupEnd();
                        return PNOL_ERR_COMM;
                    }
            } else if (ncclRecv(p, rows * ld, ncclDouble, o, g_comm.nccl, ctx->stream) != ncclSuccess) {
                ncclGroupEnd();
                return PNOL_ERR_COMM;
            }
        }
        if (ncclGroupEnd() != ncclSuccess) return PNOL_ERR_COMM;
        return PNOL_OK;
    }
    // host backend: every rank packs at most ceil(nt / P) tiles into one slot of the gather
    const int slot_tiles = (nt + P - 1) / P;
    const size_t slot = (size_t)slot_tiles * kFdTileCols * ld;
    void *sv = nullptr, *rv = nullptr;
    PNOL_CHECK(ws_get(ctx, "share_send", sizeof(double) * slot, &sv));
    PNOL_CHECK(ws_get(ctx, "share_recv", sizeof(double) * slot * P, &rv));
    double *send = (double*)sv, *recv = (double*)rv;
    std::vector<int> st, ct;
    fd_tiles_of(ncols, P, me, st, ct);
    for (size_t i = 0; i < st.size(); ++i)
        PNOL_HIP(hipMemcpyAsync(send + i * kFdTileCols * ld, buf + (size_t)st[i] * ld, sizeof(double) * ct[i] * ld,
                                hipMemcpyDeviceToDevice, ctx->stream));
    PNOL_CHECK(comm_allgather_device(ctx, send, recv, slot));
    for (int r = 0; r < P; ++r) {
        if (r == me) continue;
        fd_tiles_of(ncols, P, r, st, ct);
        for (size_t i = 0; i < st.size(); ++i)
            PNOL_HIP(hipMemcpyAsync(buf + (size_t)st[i] * ld, recv + r * slot + i * kFdTileCols * ld,
                                    sizeof(double) * ct[i] * ld, hipMemcpyDeviceToDevice, ctx->stream));
    }
    return PNOL_OK;
}

int comm_exchange(pnol_ctx* ctx, const double* sbase, double* rbase,
                  const std::function<void(int, int, std::vector<XBlock>&)>& blocks, void* stream_) {
    const int P = g_comm.nranks, me = g_comm.rank;
    if (g_comm.kind == 0 || P == 1) return PNOL_OK;
    const hipStream_t st = stream_ ? (hipStream_t)stream_ : ctx->stream;
    std::vector<XBlock> bl;
    if (g_comm.kind == 1) {
        if (!g_comm.nccl) return PNOL_ERR_COMM;
        if (ncclGroupStart() != ncclSuccess) return PNOL_ERR_COMM;
        bool ok = true;
        for (int d = 0; d < P && ok; ++d) {
            if (d == me) continue;
            blocks(me, d, bl);
            for (const XBlock& b : bl)
                if (b.count && ncclSend(sbase + b.soff, b.count, ncclDouble, d, g_comm.nccl, st) != ncclSuccess)
                    ok = false;
        }
        for (int q = 0; q < P && ok; ++q) {
            if (q == me) continue;
            blocks(q, me, bl);
            for (const XBlock& b : bl)
                if (b.count && ncclRecv(rbase + b.roff, b.count, ncclDouble, q, g_comm.nccl, st) != ncclSuccess)
                    ok = false;
        }
        if (ncclGroupEnd() != ncclSuccess || !ok) return PNOL_ERR_COMM;
        return PNOL_OK;
    }
    // host backend: every rank packs all its outgoing blocks (destinations in order) into one
    // slot of the largest rank's size; one allgather; receivers pick their blocks out.  The
    // host waits for `st` anyway (the allgather below): first for its earlier copies, so a
    // scratch regrow cannot free a buffer they still read.
    PNOL_CHECK(stream_wait(st));
    auto out_size = [&](int q) {
        size_t t = 0;
        for (int d = 0; d < P; ++d) {
            if (d == q) continue;
            blocks(q, d, bl);
            for (const XBlock& b : bl) t += b.count;
        }
        return t;
    };
    size_t slot = 1;
    for (int q = 0; q < P; ++q) slot = std::max(slot, out_size(q));
    void *sv = nullptr, *rv = nullptr;
    // (a buffer regrow synchronises the context stream: sizes settle on the first trip)
    PNOL_CHECK(ws_get(ctx, "xchg_send", sizeof(double) * slot, &sv));
    PNOL_CHECK(ws_get(ctx, "xchg_recv", sizeof(double) * slot * P, &rv));
    double *send = (double*)sv, *recv = (double*)rv;
    size_t off = 0;
    for (int d = 0; d < P; ++d) {
        if (d == me) continue;
        blocks(me, d, bl);
        for (const XBlock& b : bl) {
            if (b.count)
                PNOL_HIP(hipMemcpyAsync(send + off, sbase + b.soff, sizeof(double) * b.count, hipMemcpyDeviceToDevice,
                                        st));
            off += b.count;
        }
    }
    PNOL_CHECK(comm_allgather_device(ctx, send, recv, slot, st));
    for (int q = 0; q < P; ++q) {
        if (q == me) continue;
        off = 0;
        for (int d = 0; d < P; ++d) {
            if (d == q) continue;
            blocks(q, d, bl);
            for (const XBlock& b : bl) {
                if (d == me && b.count)
                    PNOL_HIP(hipMemcpyAsync(rbase + b.roff, recv + (size_t)q * slot + off, sizeof(double) * b.count,
                                            hipMemcpyDeviceToDevice, st));
                off += b.count;
            }
        }
    }
    return PNOL_OK;
}

int comm_allgather_int(pnol_ctx* ctx, int mine, std::vector<int>& all) {
    const int P = g_comm.nranks;
    all.assign(P, mine);
    if (g_comm.kind == 0 || P == 1) return PNOL_OK;
    std::vector<double> v(P);
    const double m = mine;
    PNOL_CHECK(comm_allgather_host(ctx, &m, v.data(), 1));
    for (int r = 0; r < P; ++r) all[r] = (int)v[r];
    return PNOL_OK;
}

int comm_allgather_host(pnol_ctx* ctx, const double* send, double* recv, size_t count) {
    if (g_comm.kind == 0) {
        std::memcpy(recv, send, sizeof(double) * count);
        return PNOL_OK;
    }
    if (g_comm.kind == 2) return g_comm.fn(send, recv, sizeof(double) * count, g_comm.user) == 0 ? PNOL_OK : PNOL_ERR_COMM;
    // RCCL: stage through device scratch
    if (!ctx) ctx = g_comm.ctx;
    void *ds = nullptr, *dr = nullptr;
    PNOL_CHECK(ws_get(ctx, "comm_send", sizeof(double) * count, &ds));
    PNOL_CHECK(ws_get(ctx, "comm_recv", sizeof(double) * count * g_comm.nranks, &dr));
    PNOL_HIP(hipMemcpyAsync(ds, send, sizeof(double) * count, hipMemcpyHostToDevice, ctx->stream));
    PNOL_CHECK(comm_allgather_device(ctx, (const double*)ds, (double*)dr, count));
    PNOL_HIP(hipMemcpyAsync(recv, dr, sizeof(double) * count * g_comm.nranks, hipMemcpyDeviceToHost, ctx->stream));
    PNOL_CHECK(stream_wait(ctx->stream));
    return PNOL_OK;
}

int comm_allgather_device(pnol_ctx* ctx, const double* send, double* recv, size_t count, void* stream_) {
    const hipStream_t st = stream_ ? (hipStream_t)stream_ : ctx->stream;
    if (g_comm.kind == 0) {
        if (send != recv) PNOL_HIP(hipMemcpyAsync(recv, send, sizeof(double) * count, hipMemcpyDeviceToDevice, st));
        return PNOL_OK;
    }
    if (g_comm.kind == 1) {
        if (!g_comm.nccl) return PNOL_ERR_COMM;
        ScopedTimer tm(ctx, "allgather", st);
        if (ncclAllGather(send, recv, count, ncclDouble, g_comm.nccl, st) != ncclSuccess) return PNOL_ERR_COMM;
        return PNOL_OK;
    }
    // host backend with device buffers: bounce through host memory
    std::vector<double> hs(count), hr(count * (size_t)g_comm.nranks);
    PNOL_HIP(hipMemcpyAsync(hs.data(), send, sizeof(double) * count, hipMemcpyDeviceToHost, st));
    PNOL_CHECK(stream_wait(st));
    if (g_comm.fn(hs.data(), hr.data(), sizeof(double) * count, g_comm.user) != 0) return PNOL_ERR_COMM;
    PNOL_HIP(hipMemcpyAsync(recv, hr.data(), sizeof(double) * hr.size(), hipMemcpyHostToDevice, st));
    PNOL_CHECK(stream_wait(st));
    return PNOL_OK;
}

// ---------------------------------------------------------------------------------------
// kernel timers
// ---------------------------------------------------------------------------------------
// mode 2: the kernels bench.py prices against a roofline or a scaling target; each timer
// costs two event records between launches (~5 us of dispatch gap each)
static bool hot_timer(const char* name) {
    for (const char* h : {"fd_jacobian", "fd_ckpt", "syrk", "exchange_J", "exchange_J_busy", "allgather", "hg",
                          "bfgs_pass"})
        if (std::strcmp(name, h) == 0) return true;
    return false;
}

ScopedTimer::ScopedTimer(pnol_ctx* ctx, const char* name, hipStream_t stream)
    : ctx_(ctx), name_(name), stream_(stream) {
    if (!ctx_ || !ctx_->timers.on) return;
    if (ctx_->timers.on == 2 && !hot_timer(name)) return;
    if (!stream_) stream_ = ctx_->stream;
    auto& pool = ctx_->timers.free_events;
    for (hipEvent_t* e : {&a_, &b_}) {
        if (!pool.empty()) {
            *e = pool.back();
            pool.pop_back();
        } else if (hipEventCreate(e) != hipSuccess) {
            a_ = b_ = nullptr;
            return;
        }
    }
    (void)hipEventRecord(a_, stream_);
}

LaunchTimer::LaunchTimer(pnol_ctx* ctx, const char* name) : ctx_(ctx), name_(name) {
    if (!ctx_ || !ctx_->timers.on) return;
    if (ctx_->timers.on == 2 && !hot_timer(name)) return;
    auto& pool = ctx_->timers.free_events;
    for (hipEvent_t* e : {&a_, &b_}) {
        if (!pool.empty()) {
            *e = pool.back();
            pool.pop_back();
        } else if (hipEventCreate(e) != hipSuccess) {
            a_ = b_ = nullptr;
            return;
        }
    }
}

LaunchTimer::~LaunchTimer() {
    if (a_) ctx_->timers.pending[name_].push_back({a_, b_});
}

ScopedTimer::~ScopedTimer() {
    if (!a_) return;
    (void)hipEventRecord(b_, stream_);
    ctx_->timers.pending[name_].push_back({a_, b_});
}

static bool timer_take(pnol_ctx* ctx, hipEvent_t* e) {
    auto& pool = ctx->timers.free_events;
    if (!pool.empty()) {
        *e = pool.back();
        pool.pop_back();
        return true;
    }
    return hipEventCreate(e) == hipSuccess;
}

hipEvent_t timer_event(pnol_ctx* ctx, const char* name, hipStream_t stream) {
    if (!ctx || !ctx->timers.on || (ctx->timers.on == 2 && !hot_timer(name))) return nullptr;
    hipEvent_t e = nullptr;
    if (!timer_take(ctx, &e)) return nullptr;
    (void)hipEventRecord(e, stream ? stream : ctx->stream);
    return e;
}

void timer_pair(pnol_ctx* ctx, const char* name, hipEvent_t a, hipEvent_t b) {
    if (!ctx) return;
    if (a && b) {
        ctx->timers.pending[name].push_back({a, b});
        return;
    }
    for (hipEvent_t e : {a, b})
        if (e) ctx->timers.free_events.push_back(e);
}

static void resolve_timers(pnol_ctx* ctx) {
    for (auto& kv : ctx->timers.pending) {
        auto& acc = ctx->timers.done[kv.first];
        for (auto& ev : kv.second) {
            float ms = 0.f;
            (void)hipEventSynchronize(ev.second);
            (void)hipEventSynchronize(ev.first);
            if (hipEventElapsedTime(&ms, ev.first, ev.second) == hipSuccess) {
                acc.first += ms > 0.f ? ms : 0.f;   // a cross-stream pair may end before it starts
                acc.second += 1;
            }
            ctx->timers.free_events.push_back(ev.first);
            ctx->timers.free_events.push_back(ev.second);
        }
        kv.second.clear();
    }
}

// ---------------------------------------------------------------------------------------
// default context for the C++ drop-in classes
// ---------------------------------------------------------------------------------------
static pnol_ctx* g_default = nullptr;
static std::mutex g_default_mu;
static int g_default_dev = -1;   // pnol_set_default_device

pnol_ctx* default_ctx_or_null() {
    std::lock_guard<std::mutex> lk(g_default_mu);
    if (g_default) return g_default;
    int count = 0;
    if (pnol_device_count(&count) != PNOL_OK || count == 0) return nullptr;
    int dev = 0;
    if (g_default_dev >= 0) dev = g_default_dev;
    else if (const char* e = std::getenv("PNOL_DEVICE")) dev = std::atoi(e);
    else {
        // node-local rank of torchrun, MPICH / Intel MPI (hydra) or Open MPI
        for (const char* k : {"LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK"}) {
            const int l = env_int(k, -1);
            if (l >= 0) {
                dev = l % count;
                break;
            }
        }
    }
    pnol_ctx* c = nullptr;
    if (pnol_ctx_create(dev, &c) != PNOL_OK) return nullptr;
    g_default = c;
    return g_default;
}

// Host <-> device copies of the solvers' small vectors (x, sigma, residuals): through a
// pinned staging buffer, so the DMA engine copies directly instead of the runtime's pageable
// bounce path.  Large copies (> 64 MiB) go direct.
void* pinned_stage(pnol_ctx* ctx, size_t bytes) {
    constexpr size_t kMaxStage = 64u << 20;
    if (bytes > kMaxStage) return nullptr;
    if (ctx->pinned_bytes < bytes) {
        if (ctx->pinned) (void)hipHostFree(ctx->pinned);
        ctx->pinned = nullptr;
        ctx->pinned_bytes = 0;
        size_t cap = 64 * 1024;
        while (cap < bytes) cap *= 2;
        if (hipHostMalloc(&ctx->pinned, cap, hipHostMallocDefault) != hipSuccess) {
            ctx->pinned = nullptr;
            return nullptr;
        }
        ctx->pinned_bytes = cap;
    }
    return ctx->pinned;
}

}  // namespace pnol

using namespace pnol;

extern "C" {

const char* pnol_status_string(int s) {
    switch (s) {
        case PNOL_OK: return "ok";
        case PNOL_ERR_ARG: return "invalid argument";
        case PNOL_ERR_HIP: return "HIP runtime error";
        case PNOL_ERR_NOMEM: return "out of device memory";
        case PNOL_ERR_NODEVICE: return "no gfx950 (MI355X) device visible";
        case PNOL_ERR_SINGULAR: return "singular system";
        case PNOL_ERR_COMM: return "communicator error";
        case PNOL_ERR_UNSUPPORTED: return "unsupported";
        case PNOL_ERR_TIMEOUT: return "device wait timed out (the tile Cholesky, after its relaunches)";
        default: return "unknown status";
    }
}

int pnol_version(void) { return PNOL_AMD_VERSION; }

int pnol_device_count(int* count) {
    if (!count) return PNOL_ERR_ARG;
    *count = 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return PNOL_OK;
    int c = 0;
    for (int d = 0; d < n; ++d)
        if (is_gfx950(d)) ++c;
    *count = c;
    return PNOL_OK;
}

int pnol_ctx_create(int device, pnol_ctx** out) {
    if (!out) return PNOL_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n || !is_gfx950(device))
        return PNOL_ERR_NODEVICE;
    PNOL_HIP(hipSetDevice(device));
    auto* c = new pnol_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return PNOL_ERR_HIP;
    }
    c->stream = c->own_stream;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cu = prop.multiProcessorCount;
    *out = c;
    return PNOL_OK;
}

int pnol_ctx_destroy(pnol_ctx* ctx) {
    if (!ctx) return PNOL_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& kv : ctx->ws.bufs)
        if (kv.second.first) (void)hipFree(kv.second.first);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    if (ctx->aux_stream) {
        (void)hipStreamSynchronize(ctx->aux_stream);
        (void)hipStreamDestroy(ctx->aux_stream);
    }
    for (hipEvent_t e : ctx->aux_events) (void)hipEventDestroy(e);
    if (ctx->comm_stream) {
        (void)hipStreamSynchronize(ctx->comm_stream);
        (void)hipStreamDestroy(ctx->comm_stream);
    }
    for (hipEvent_t e : ctx->phase_events) (void)hipEventDestroy(e);
    if (ctx->comm_done) (void)hipEventDestroy(ctx->comm_done);
    for (auto& kv : ctx->timers.pending)
        for (auto& ev : kv.second) {
            (void)hipEventDestroy(ev.first);
            (void)hipEventDestroy(ev.second);
        }
    for (hipEvent_t e : ctx->timers.free_events) (void)hipEventDestroy(e);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    (void)hipGetLastError();   // a failed clean-up call must not surface at the next launch check
    if (ctx == g_default) g_default = nullptr;
    delete ctx;
    return PNOL_OK;
}

int pnol_ctx_synchronize(pnol_ctx* ctx) {
    if (!ctx) return PNOL_ERR_ARG;
    PNOL_CHECK(stream_wait(ctx->stream));
    return PNOL_OK;
}

int pnol_ctx_get_stream(pnol_ctx* ctx, void** s) {
    if (!ctx || !s) return PNOL_ERR_ARG;
    *s = (void*)ctx->stream;
    return PNOL_OK;
}

int pnol_ctx_set_stream(pnol_ctx* ctx, void* s) {
    if (!ctx) return PNOL_ERR_ARG;
    ctx->stream = s ? (hipStream_t)s : ctx->own_stream;
    return PNOL_OK;
}

int pnol_ctx_device(pnol_ctx* ctx, int* device) {
    if (!ctx || !device) return PNOL_ERR_ARG;
    *device = ctx->device;
    return PNOL_OK;
}

int pnol_default_ctx(pnol_ctx** out) {
    if (!out) return PNOL_ERR_ARG;
    *out = default_ctx_or_null();
    return *out ? PNOL_OK : PNOL_ERR_NODEVICE;
}

int pnol_ctx_enable_timers(pnol_ctx* ctx, int on) {
    if (!ctx) return PNOL_ERR_ARG;
    ctx->timers.on = on == 2 ? 2 : (on != 0 ? 1 : 0);
    // events for the timers made up front: a hipEventCreate between a trip's launches sat on the
    // host's path to the next FD launch (events return to the pool when the timers are read)
    if (ctx->timers.on) {
        PNOL_HIP(hipSetDevice(ctx->device));
        auto& pool = ctx->timers.free_events;
        while (pool.size() < 512) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) break;
            pool.push_back(e);
        }
    }
    return PNOL_OK;
}

int pnol_ctx_reset_timers(pnol_ctx* ctx) {
    if (!ctx) return PNOL_ERR_ARG;
    resolve_timers(ctx);
    ctx->timers.done.clear();
    return PNOL_OK;
}

int pnol_ctx_timer(pnol_ctx* ctx, const char* name, double* total_ms, int* count) {
    if (!ctx || !name) return PNOL_ERR_ARG;
    resolve_timers(ctx);
    auto it = ctx->timers.done.find(name);
    if (total_ms) *total_ms = it == ctx->timers.done.end() ? 0.0 : it->second.first;
    if (count) *count = it == ctx->timers.done.end() ? 0 : it->second.second;
    return PNOL_OK;
}

int pnol_malloc(pnol_ctx* ctx, size_t bytes, void** dptr) {
    if (!ctx || !dptr) return PNOL_ERR_ARG;
    PNOL_HIP(hipSetDevice(ctx->device));
    if (hipMalloc(dptr, bytes ? bytes : 16) != hipSuccess) return PNOL_ERR_NOMEM;
    return PNOL_OK;
}

int pnol_free(pnol_ctx* ctx, void* dptr) {
    if (!ctx) return PNOL_ERR_ARG;
    if (dptr) PNOL_HIP(hipFree(dptr));
    return PNOL_OK;
}

int pnol_memcpy_h2d(pnol_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx || (!dst && bytes) || (!src && bytes)) return PNOL_ERR_ARG;
    if (!bytes) return PNOL_OK;
    if (void* st = pinned_stage(ctx, bytes)) {
        std::memcpy(st, src, bytes);
        PNOL_HIP(hipMemcpyAsync(dst, st, bytes, hipMemcpyHostToDevice, ctx->stream));
    } else {
        PNOL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    }
    PNOL_CHECK(stream_wait(ctx->stream));
    return PNOL_OK;
}

int pnol_memcpy_d2h(pnol_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx || (!dst && bytes) || (!src && bytes)) return PNOL_ERR_ARG;
    if (!bytes) return PNOL_OK;
    if (void* st = pinned_stage(ctx, bytes)) {
        PNOL_HIP(hipMemcpyAsync(st, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
        PNOL_CHECK(stream_wait(ctx->stream));
        std::memcpy(dst, st, bytes);
    } else {
        PNOL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
        PNOL_CHECK(stream_wait(ctx->stream));
    }
    return PNOL_OK;
}

int pnol_host_alloc(void** p, size_t bytes) {
    if (!p) return PNOL_ERR_ARG;
    *p = nullptr;
    PNOL_HIP(hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault));
    return PNOL_OK;
}

int pnol_host_free(void* p) {
    if (p) PNOL_HIP(hipHostFree(p));
    return PNOL_OK;
}

int pnol_memcpy_d2h_async(pnol_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx || (!dst && bytes) || (!src && bytes)) return PNOL_ERR_ARG;
    if (bytes) PNOL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    return PNOL_OK;
}

struct pnol_event {
    hipEvent_t e = nullptr;
    int device = 0;
};

int pnol_event_create(pnol_ctx* ctx, pnol_event** out) {
    if (!ctx || !out) return PNOL_ERR_ARG;
    PNOL_HIP(hipSetDevice(ctx->device));
    auto* ev = new pnol_event();
    ev->device = ctx->device;
    if (hipEventCreateWithFlags(&ev->e, hipEventDisableTiming) != hipSuccess) {
        delete ev;
        return PNOL_ERR_HIP;
    }
    *out = ev;
    return PNOL_OK;
}

int pnol_event_record(pnol_ctx* ctx, pnol_event* ev) {
    if (!ctx || !ev) return PNOL_ERR_ARG;
    PNOL_HIP(hipEventRecord(ev->e, ctx->stream));
    return PNOL_OK;
}

// Busy-polls: the host wakes as soon as the event completes (a blocking wait returns
// tens of microseconds late, which the LM loop pays on every trip).
int pnol_event_wait(pnol_event* ev) {
    if (!ev) return PNOL_ERR_ARG;
    return event_wait(ev->e);
}

int pnol_event_destroy(pnol_event* ev) {
    if (!ev) return PNOL_ERR_ARG;
    (void)hipSetDevice(ev->device);
    (void)hipEventDestroy(ev->e);
    (void)hipGetLastError();
    delete ev;
    return PNOL_OK;
}

int pnol_comm_unique_id(char id[128]) {
    if (!id) return PNOL_ERR_ARG;
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return PNOL_ERR_COMM;
    std::memcpy(id, &u, 128);
    return PNOL_OK;
}

int pnol_comm_init_rccl(pnol_ctx* ctx, int nranks, int rank, const char id[128]) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return PNOL_ERR_ARG;
    pnol_comm_finalize();
    PNOL_HIP(hipSetDevice(ctx->device));
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    ncclComm_t c;
    if (ncclCommInitRank(&c, nranks, u, rank) != ncclSuccess) return PNOL_ERR_COMM;
    g_comm.kind = 1;
    g_comm.nranks = nranks;
    g_comm.rank = rank;
    g_comm.nccl = c;
    g_comm.ctx = ctx;
    return PNOL_OK;
}

int pnol_comm_init_host(int nranks, int rank, pnol_host_allgather_fn fn, void* user) {
    if (!fn || nranks < 1 || rank < 0 || rank >= nranks) return PNOL_ERR_ARG;
    pnol_comm_finalize();
    g_comm.kind = 2;
    g_comm.nranks = nranks;
    g_comm.rank = rank;
    g_comm.fn = fn;
    g_comm.user = user;
    return PNOL_OK;
}

int pnol_comm_finalize(void) {
    if (g_comm.kind == 1 && g_comm.nccl) ncclCommDestroy(g_comm.nccl);
    g_comm = CommState();
    return PNOL_OK;
}

int pnol_comm_set_launcher_hook(pnol_launcher_hook_fn fn) {
    std::lock_guard<std::mutex> lk(g_launch_mu);
    g_launch_hook = fn;
    g_launch_bound = false;
    return PNOL_OK;
}

int pnol_comm_bind_launcher(void) { return comm_bind_launcher(); }

int pnol_launcher_world_size(void) { return launcher_world_size(); }

int pnol_set_default_device(int device) {
    if (device < 0) return PNOL_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_default_mu);
    if (g_default) return g_default->device == device ? PNOL_OK : PNOL_ERR_ARG;
    g_default_dev = device;
    return PNOL_OK;
}

int pnol_comm_size(int* nranks, int* rank) {
    if (!nranks || !rank) return PNOL_ERR_ARG;
    *nranks = g_comm.nranks;
    *rank = g_comm.rank;
    return PNOL_OK;
}

int pnol_comm_allgather_d(pnol_ctx* ctx, const double* send, double* recv, size_t count) {
    if (!ctx || !send || !recv) return PNOL_ERR_ARG;
    return comm_allgather_device(ctx, send, recv, count);
}

void pnol_block_range(int ncols, int nranks, int rank, int* begin, int* count) {
    block_range(ncols, nranks, rank, begin, count);
}

int pnol_fd_tiles(int ncols, int nranks, int rank, int* start, int* count, int cap) {
    if (ncols < 0 || nranks < 1 || rank < 0 || rank >= nranks) return -PNOL_ERR_ARG;
    std::vector<int> st, ct;
    fd_tiles_of(ncols, nranks, rank, st, ct);
    for (size_t i = 0; i < st.size() && (int)i < cap; ++i) {
        if (start) start[i] = st[i];
        if (count) count[i] = ct[i];
    }
    return (int)st.size();
}

int pnol_comm_share_fd_rows_d(pnol_ctx* ctx, double* buf, int ld, int ncols) {
    if (!ctx || !buf || ld < 1 || ncols < 0) return PNOL_ERR_ARG;
    return comm_share_rows(ctx, buf, (size_t)ld, ncols);
}

}  // extern "C"
