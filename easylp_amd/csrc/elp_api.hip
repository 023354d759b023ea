// elp_api.hip -- host driver and C ABI (include/easylp_hip.h).
//
// The host never looks at the LP data during the solve: it enqueues
// `sync_every` iterations (7-8 kernels each) on one HIP stream, then reads
// the 300-byte device control block once to decide what happens next
// (refactor, phase switch, stop).  This mirrors the loop of
// oracle/elp_oracle.c run_phase() and the status mapping of
// /root/reference/R/class.R:279-295.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <map>
#include <unordered_map>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/easylp_hip.h"
#include "elp_comm.h"
#include "elp_internal.h"

using namespace elp;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                    \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess)                                                           \
            return fail(ELP_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));  \
    } while (0)

double now_s() {
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct elp_handle {
    double dbg_enqueue = 0.0, dbg_wait = 0.0;  // ELP_DEBUG_ENQUEUE
    int64_t m = 0, n = 0;        // global problem size
    int64_t col0 = 0, nloc = 0;  // this rank's column shard
    elp_control ctl{};
    int dev = 0;
    hipStream_t st = nullptr;
    Dev d{};
    double* A_owned = nullptr;
    // large buffers kept across reloads of the handle (a fresh hipMalloc of
    // tens of GB right after a hipFree of the same size measured 0.4-3.7 s)
    double* keep_A = nullptr;
    size_t keep_A_bytes = 0, A_owned_bytes = 0;
    size_t w_cap = 0;
    bool loaded = false, done = false;
    int maximize = 0;
    int phase = 2;
    bool any_art = false;
    int32_t final_status = ELP_SUBOPTIMAL;
    DevCtl* hctl = nullptr;  // pinned mirror
    int k_sync = 0, ny_sync = 0, since_refactor_sync = 0;
    std::vector<double> obj_h;  // global objective (for the objective value)
    std::vector<int32_t> dir_h;  // row directions and rhs (sensitivity report, MIP nodes)
    std::vector<double> rhs_h;
    std::vector<double> lo_h, up_h;  // column bounds as loaded (MIP root)
    std::vector<int32_t> is_int;     // integer columns (elp_set_int); empty: LP
    bool in_bnb = false;             // node reloads keep is_int / root bounds
    int64_t bnb_iter_left = 0;       // branch and bound: LP iterations left (max_iter > 0)
    bool mip = false;                // the last elp_solve ran branch and bound
    int64_t mip_nodes = 0, mip_iters = 0;
    elp_stats stats{};
    double t_solve_start = 0.0;
    bool timing_started = false;
    int64_t trace_cap = 0;
    elp::Comm comm;  // multi-GPU (world 1 = no-op)
    std::vector<hipEvent_t> ev;  // pricing-kernel timing pairs (profile mode)
    int64_t prof_chunks = 0;     // chunks seen by ELP_PROFILE_SAMPLE
    int32_t* d_flag = nullptr;   // one int for cross-rank decisions
    int64_t ar_rows = 0;         // AR capacity in rows (grown at polls)
    int64_t shape_m = -1, shape_n = -1;  // the previous load's shape (reloads start at its grown capacities)
    bool shape_csc = false;
    bool replicated = false;     // sharded, every rank holds all of A (Dev::Afull)
    bool csc = false;            // A given in CSC (elp_load_csc)
    int64_t mb_epoch = 0;        // loads so far (xGMI mailbox sequence epoch)
    // ELP_STAMPS debug: k_ratio phase stamps, summed over polled chunks
    std::vector<double> stamp_sum;
    int64_t stamp_n = 0;
    // single-process multi-device (elp_control.ngpu > 1): this handle drives one
    // rank handle per device (see "ngpu" below); empty for an ordinary handle
    std::vector<elp_handle*> ranks;
    std::vector<int> rank_dev;
    std::unique_ptr<elp::ThreadGroup> tgroup;  // ranks sharing a device
    std::vector<elp::ThreadRank> tranks;
    std::vector<double*> peer_A;  // elp_load_dense_device: A copied to the other devices
    std::vector<size_t> peer_A_bytes;  // (elements held by each copy)
    bool broken = false;          // a rank failed and the RCCL communicators were aborted
    int32_t sel_cap = 0;          // Dev::sel_cap (rank handles sharing a device)
    // buffers replaced by a growth at a poll, freed at the next load / destroy
    // (ranks sharing a device: hipFree waits for the device to drain, and the
    // other ranks' select kernels spin on this rank's next mailbox record)
    std::vector<void*> retired;
    // a warm-started B&B node's bounds (reload_bounds_warm), n each: allocated at
    // the first node and kept, so no node allocates or frees (a hipFree would
    // wait for peers spinning on this rank's record when ranks share a device)
    double* warm_lo = nullptr;
    double* warm_up = nullptr;
    // the load's staging of the scaled bounds and rhs (load_common: lo, up | rhs),
    // allocated with the other buffers -- a hipFree per load waited for the device
    double* ld_stage = nullptr;
    // buffers of the last load kept for the next one (free_dev on a reload):
    // alloc_all's allocations by size; a reload of the same shape takes them
    // back instead of ~80 hipFree + hipMalloc pairs (1.8 ms at 5000 x 50000)
    std::unordered_map<void*, size_t> asize;
    std::multimap<size_t, void*> pool;
    // scaling (elp_control.scaling): the solver works on A~ = 2^srow A 2^scol
    // (exponents per row and per GLOBAL column; empty: unscaled)
    std::vector<int32_t> srow_h, scol_h;
    int64_t kcap = 0;  // bump capacity: AS m x kcap, Minv / MinvT kcap x kcap (grown at polls)

    bool dual_used = false;  // the last load's phase 1 is the dual simplex (phase 3)
    elp::ResOut* d_resout = nullptr;  // the resident solver's exit record, then x (RES_PIN_X: one copy back)
    size_t res_lds_max = 0;           // LDS one workgroup may allocate (0: not queried yet)
    // the resident solver's exit: the structurals' values (scaled) brought back
    // with the control block; res_fresh: hctl and res_x equal the device's
    // (nothing ran since), so the next node, elp_get_stats and
    // elp_get_solution skip their round trips; res_warm: the next resident
    // launch runs the node warm start first
    double* d_resx = nullptr;  // (inside d_resout's allocation)
    std::vector<double> res_x;
    // pinned host block of the resident exchanges: [ResOut][x: n][node lo: n][node up: n]
    // (pageable copies of these few bytes block the host for the whole transfer)
    char* res_pin = nullptr;
    bool res_fresh = false;
    int32_t res_warm = 0;
    // ctl_fresh: hctl equals the device's control block (the load's last
    // transfer wrote it), so run_loop skips its refresh
    bool ctl_fresh = false;
    std::vector<double> mip_x;   // branch and bound: the incumbent (elp_get_solution)
};

// elp_control.simplex = 0 (include/easylp_hip.h): lp_solve's default,
// SIMPLEX_DUAL_PRIMAL, wherever the dual phase exists (dual_phase1)
#define ELP_SIMPLEX_DEFAULT ELP_SIMPLEX_DUAL_PRIMAL

extern "C" void elp_default_control(elp_control* c) {
    std::memset(c, 0, sizeof(*c));
    c->tol_primal = 1e-9;
    c->tol_dual = 1e-9;
    c->tol_pivot = 1e-9;
    c->infinity = 1e30;
    c->time_limit = 0.0;
    c->max_iter = 0;
    c->refactor_period = 250;  // lp_solve's default set_maxpivot
    c->degen_switch = 50;
    c->device = 0;
    c->sync_every = 32;
    c->verbose = 0;
    c->pricing = ELP_PRICE_DEVEX;
    c->ngpu = 1;
    c->scaling = ELP_SCALE_GEOMETRIC | ELP_SCALE_EQUILIBRATE;  // lp_solve's default scaling
    c->tol_singular = 1e-13;
    c->mailbox_timeout = 2.0;
}

extern "C" const char* elp_last_error(void) { return g_err.c_str(); }
extern "C" int32_t elp_abi_version(void) { return ELP_ABI_VERSION; }

static void release_kept(elp_handle* h) {
    if (h->keep_A) (void)hipFree(h->keep_A);
    h->keep_A = nullptr;
    h->keep_A_bytes = 0;
}

static void drain_pool(elp_handle* h) {
    for (auto& kv : h->pool) (void)hipFree(kv.second);
    h->pool.clear();
}

// keep_big: a reload -- A's copy stays allocated for the next load, the other
// buffers go to the handle's pool (dalloc inside alloc_all takes them back)
static void free_dev(elp_handle* h, bool keep_big = false) {
    Dev& d = h->d;
    if (keep_big) {
        release_kept(h);
        h->keep_A = h->A_owned;
        h->keep_A_bytes = h->A_owned ? h->A_owned_bytes : 0;
        h->A_owned = nullptr;
    }
    auto release = [&](void* p) {
        const auto it = h->asize.find(p);
        if (keep_big && it != h->asize.end()) h->pool.emplace(it->second, p);
        else (void)hipFree(p);
        if (it != h->asize.end()) h->asize.erase(it);
    };
    void* ptrs[] = {h->A_owned, d.AR,  d.AS,    d.Minv,  d.W0,   d.W1,    d.b,     d.obj,
                    d.lb,       d.ub,  d.cost,  d.xval,  d.asgn, d.xr,    d.xs,    d.y,
                    d.t,        d.acol, d.aR,   d.alS,   d.alU,  d.zz,    d.zpart, d.vrow,
                    d.vvec,     d.colA, d.rhs,  d.vstat, d.cover, d.rpos, d.Rl,    d.Sl,
                    d.Yl,  d.ypos,  d.perm,  d.pivstep, d.nzlist, d.nzcount, d.nzchunk,
                    d.cand,     d.pstamp, d.ctl, d.trace, d.MinvT, d.yy, d.blockmin, d.rcand, d.rcnt,
                    d.pkt, d.objg, d.ract, d.cand_xchg, h->d_flag, d.cS, d.slo, d.shi, d.rlo, d.rhi,
                    (void*)d.cptr, (void*)d.rind, (void*)d.cval, (void*)d.rptr, (void*)d.cind,
                    (void*)d.rval, d.qcol, d.qz, d.spos, d.dstamp, d.rowvs, d.yvs, d.dw, d.dprev, (void*)d.srow,
                    (void*)d.scol, d.rhoR, d.rr, d.dchz, d.dcand, d.dcnt, d.dcomp, d.dalive, d.dflip,
                    d.dflipdx, d.aF, d.fS, d.ddw != d.dw ? (void*)d.ddw : nullptr, d.dsend, d.drecv,
                    d.afs, d.afl, d.aflv, d.ptst, d.ptgrid, h->ld_stage};
    for (void* p : ptrs)
        if (p) release(p);
    if (!keep_big) drain_pool(h);
    for (void* p : h->retired) (void)hipFree(p);
    h->retired.clear();
    if (h->warm_lo) (void)hipFree(h->warm_lo);
    if (h->warm_up) (void)hipFree(h->warm_up);
    h->warm_lo = h->warm_up = nullptr;
    h->A_owned = nullptr;
    h->d_flag = nullptr;
    h->ld_stage = nullptr;
    h->w_cap = 0;  // (W0 / W1 went with the rest)
    d = Dev{};
    if (h->hctl && !keep_big) {  // (a reload keeps the pinned control-block copy)
        (void)hipHostFree(h->hctl);
        h->hctl = nullptr;
    }
}

// a buffer a growth replaced (see elp_handle::retired)
static void retire(elp_handle* h, void* p) {
    if (!p) return;
    h->asize.erase(p);  // (never pooled: a growth replaced it)
    if (h->sel_cap > 0) h->retired.push_back(p);
    else (void)hipFree(p);
}

// the handle whose alloc_all is running on this thread (ngpu ranks load on
// threads of their own): dalloc then draws on and records into its pool
static thread_local elp_handle* t_alloc_h = nullptr;
template <class T>
static hipError_t dalloc(T** p, size_t count) {
    const size_t bytes = (count ? count : 1) * sizeof(T);
    elp_handle* h = t_alloc_h;
    if (!h) return hipMalloc((void**)p, bytes);
    const auto it = h->pool.find(bytes);
    if (it != h->pool.end()) {
        *p = static_cast<T*>(it->second);
        h->pool.erase(it);
    } else {
        const hipError_t e = hipMalloc((void**)p, bytes);
        if (e != hipSuccess) return e;
    }
    h->asize[*p] = bytes;
    return hipSuccess;
}

// a buffer of `bytes`, the kept one when it is exactly that size
static hipError_t take_or_alloc(double** p, size_t bytes, double** keep, size_t* keep_bytes) {
    if (*keep && *keep_bytes == bytes) {
        *p = *keep;
        *keep = nullptr;
        *keep_bytes = 0;
        return hipSuccess;
    }
    if (*keep) (void)hipFree(*keep);
    *keep = nullptr;
    *keep_bytes = 0;
    return hipMalloc((void**)p, bytes ? bytes : sizeof(double));  // (m = 0: kernels read element 0)
}

// ---------------------------------------------------------------- spares
// A destroyed one-GPU handle leaves its stream, its device buffers (by size),
// its pinned blocks and its copy of A for the next elp_create on the same
// device (R's flow: one handle per easylp$solve(), make.lp ... finalize): a
// stream creation costs 0.4-8 ms and a small LP's ~45 buffers ~0.13 ms, more
// than the solve.  Bounded: SPARE_MAX handles' worth, SPARE_BYTES of device
// memory in all; ELP_NO_SPARE=1 turns it off.  The next load takes buffers
// of the sizes it needs (alloc_all's pool) and frees the rest.
struct Spare {
    int dev = 0;
    hipStream_t st = nullptr;
    std::multimap<size_t, void*> pool;
    size_t bytes = 0;
    double* keep_A = nullptr;
    size_t keep_A_bytes = 0;
    DevCtl* hctl = nullptr;
    ResOut* resout = nullptr;
    int64_t resx_n = 0;  // (resout holds the record and x: sized by n)
    char* respin = nullptr;
};
static std::mutex g_spare_mu;
static std::vector<Spare> g_spares;
constexpr int SPARE_MAX = 4;
constexpr size_t SPARE_BYTES = (size_t)1 << 30;
static bool spares_on() {
    static const bool on = [] {
        const char* e = std::getenv("ELP_NO_SPARE");
        return !(e && std::atoi(e) != 0);
    }();
    return on;
}
static void spare_free(Spare& sp) {
    (void)hipSetDevice(sp.dev);
    for (auto& kv : sp.pool) (void)hipFree(kv.second);
    if (sp.keep_A) (void)hipFree(sp.keep_A);
    if (sp.hctl) (void)hipHostFree(sp.hctl);
    if (sp.resout) (void)hipFree(sp.resout);
    if (sp.respin) (void)hipHostFree(sp.respin);
    if (sp.st) (void)hipStreamDestroy(sp.st);
}

// ---------------------------------------------------------------- ngpu
// Single-process multi-device (elp_control.ngpu = P > 1; SURVEY.md 8b
// "Threading": the R caller stays one synchronous process): the handle the
// caller holds drives P rank handles, one per device, each the column-sharded
// solver of one rank (elp_comm_* semantics).  Every API call runs on all ranks
// at once -- one host thread per rank (RCCL ranks: the calling thread watches
// them; in-process ranks: rank 0 runs on the calling thread) -- and returns
// when all are done.  Ranks on distinct devices share an RCCL
// communicator from ncclCommInitAll (xGMI); ranks that share a device (fewer
// devices than P, e.g. a one-GPU box) use the in-process ThreadGroup.
static bool is_group(const elp_handle* h) { return h && !h->ranks.empty(); }

// collective = false: the call issues no collective (elp_set_int, elp_set_trace,
// the ngpu elp_sensitivity parts), so a failing rank never strands a peer and
// nothing is aborted.
// Otherwise a rank failure releases the peers that wait in a collective: the
// in-process transport fails its waiters at once (and is reset at the next
// call); RCCL communicators (distinct devices) are aborted -- for good: later
// calls fail ELP_E_STATE -- only when a peer is still running a grace period
// after the failure, i.e. actually waiting for the failed rank (a uniform
// argument / state error returns on every rank before any collective, and
// leaves the handle usable: ADVICE r03).
template <class F>
static int fan_out(elp_handle* g, F&& f, bool collective = true) {
    if (g->broken)
        return fail(ELP_E_STATE, "ngpu handle: a rank failed earlier and the communicators were aborted; "
                                 "destroy the handle");
    const int P = (int)g->ranks.size();
    if (g->tgroup) g->tgroup->reset();
    std::vector<int> rc(P, 0);
    std::vector<std::string> err(P);
    std::atomic<int> first{-1};
    std::mutex mu;
    std::condition_variable cv;
    int running = P;
    auto run = [&](int r) {
        rc[r] = f(g->ranks[r], r);
        if (rc[r] < 0) {
            err[r] = g_err;
            int none = -1;
            first.compare_exchange_strong(none, r);
            if (collective && g->tgroup) g->tgroup->abort();
        }
        std::lock_guard<std::mutex> lk(mu);
        --running;
        cv.notify_all();
    };
    // RCCL ranks (distinct devices): every rank on a worker thread and the
    // calling thread the watchdog -- rank 0 itself may be the one blocked in a
    // collective for a failed peer, and only an abort from outside releases it
    // (ADVICE r04); otherwise rank 0 runs on the calling thread
    const bool watch = collective && !g->tgroup;
    std::vector<std::thread> th;
    th.reserve((size_t)P);
    for (int r = watch ? 0 : 1; r < P; ++r) th.emplace_back(run, r);
    if (!watch) run(0);
    if (watch) {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            if (running == 0) break;
            if (first.load() < 0) {
                cv.wait(lk);
                continue;
            }
            // a rank failed: give the others the mailbox timeout to return on their own
            const double grace = std::max(1.0, g->ctl.mailbox_timeout);
            if (cv.wait_for(lk, std::chrono::duration<double>(grace), [&] { return running == 0; })) break;
            lk.unlock();
            for (elp_handle* rh : g->ranks) rh->comm.abort_rccl();
            g->broken = true;
            break;
        }
    }
    for (auto& t : th) t.join();
    const int r = first.load();
    if (r >= 0) return fail(rc[r], "rank " + std::to_string(r) + ": " + err[r]);
    return rc[0];
}

static void destroy_group(elp_handle* g) {
    for (size_t r = 0; r < g->peer_A.size(); ++r)
        if (g->peer_A[r]) {
            (void)hipSetDevice(g->rank_dev[r]);
            (void)hipFree(g->peer_A[r]);
        }
    g->peer_A.clear();
    for (elp_handle* r : g->ranks)
        if (r) elp_destroy(r);
    g->ranks.clear();
    g->tgroup.reset();
}

// ngpu: the per-iteration min-loc over a direct peer mailbox.
// One process drives every rank, so no IPC: each rank's mailbox is uncached
// memory on its own device, every device enables peer access to every other
// one, and each rank gets a device array of the P raw mailbox pointers -- the
// same store / poll protocol as the multi-process mailbox (p2p_exchange).  The
// P probes run concurrently (one per rank stream); only when every round trip
// arrives do the ranks adopt the mailboxes, else everything is released and
// the collective stays (returns 0 either way; errors of the set-up are not
// fatal).  Ranks that share a device (the one-GPU test box) use same-device
// pointers; their streams must land on distinct hardware queues, which the
// probe checks (spinning kernels behind each other on one queue never meet).
static void enable_group_p2p(elp_handle* g) {
    const int P = (int)g->ranks.size();
    if (P > 64 || g->ctl.exchange == 1) return;
    const size_t rec = sizeof(MboxRec), bytes = 2 * (size_t)P * rec;
    std::vector<void*> mb(P, nullptr);
    std::vector<void**> dp(P, nullptr);
    std::vector<int32_t*> dok(P, nullptr);
    bool ok = true;
    for (int r = 0; r < P && ok; ++r)
        for (int t = 0; t < P && ok; ++t) {
            const int a = g->rank_dev[r], b = g->rank_dev[t];
            if (a == b) continue;
            int can = 0;
            if (hipSetDevice(a) != hipSuccess || hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) {
                ok = false;
                break;
            }
            const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) ok = false;
            (void)hipGetLastError();
        }
    for (int r = 0; r < P && ok; ++r) {
        ok = hipSetDevice(g->rank_dev[r]) == hipSuccess &&
             hipExtMallocWithFlags(&mb[r], bytes, hipDeviceMallocUncached) == hipSuccess &&
             hipMemset(mb[r], 0, bytes) == hipSuccess && hipMalloc((void**)&dok[r], 2 * sizeof(int32_t)) == hipSuccess &&
             hipMemset(dok[r], 0, 2 * sizeof(int32_t)) == hipSuccess;
    }
    for (int r = 0; r < P && ok; ++r) {
        ok = hipSetDevice(g->rank_dev[r]) == hipSuccess && hipMalloc((void**)&dp[r], sizeof(void*) * P) == hipSuccess &&
             hipMemcpy(dp[r], mb.data(), sizeof(void*) * P, hipMemcpyHostToDevice) == hipSuccess;
    }
    if (ok) {
        // a probe round trip takes microseconds once every kernel runs: a short
        // limit keeps a doomed set-up (shared hardware queues) cheap
        const double secs = std::min(g->ctl.mailbox_timeout, 0.5);
        int launched = 0;
        for (int r = 0; r < P && ok; ++r, ++launched)
            ok = hipSetDevice(g->rank_dev[r]) == hipSuccess &&
                 launch_mbox_probe((void* const*)dp[r], mb[r], P, r, (int64_t)rec, dok[r],
                                   (unsigned long long)(secs * 1e8), g->ranks[r]->st) == hipSuccess;
        for (int r = 0; r < launched; ++r) {  // every launched probe drains (bounded by its limit)
            int32_t v[2] = {0, 0};
            const bool got = hipSetDevice(g->rank_dev[r]) == hipSuccess &&
                             hipStreamSynchronize(g->ranks[r]->st) == hipSuccess &&
                             hipMemcpy(v, dok[r], sizeof(v), hipMemcpyDeviceToHost) == hipSuccess;
            ok = ok && got && v[0] == 1;
            if (got && v[0] == 1) g->ranks[r]->comm.rtt_us = mbox_rtt_us(v[1]);
        }
    }
    for (int r = 0; r < P; ++r) {
        (void)hipSetDevice(g->rank_dev[r]);
        if (dok[r]) (void)hipFree(dok[r]);
        if (ok) {
            g->ranks[r]->comm.adopt_p2p(mb[r], dp[r]);
        } else {
            if (mb[r]) (void)hipFree(mb[r]);
            if (dp[r]) (void)hipFree(dp[r]);
        }
    }
    (void)hipGetLastError();
}

static int create_group(elp_handle* g) {
    const int P = g->ctl.ngpu;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(ELP_E_HIP, "elp_create: no HIP device");
    g->rank_dev.resize(P);
    for (int r = 0; r < P; ++r) g->rank_dev[r] = (g->ctl.device + r) % ndev;
    const bool distinct = P <= ndev && !std::getenv("ELP_NGPU_THREADS");
    g->ranks.assign(P, nullptr);
    for (int r = 0; r < P; ++r) {
        elp_control c = g->ctl;
        c.ngpu = 1;
        c.device = g->rank_dev[r];
        const int rc = elp_create(&g->ranks[r], g->m, g->n, &c);
        if (rc) return rc;
    }
    if (distinct) {
        std::vector<void*> comms;
        int rc = Comm::init_all(comms, g->rank_dev);
        if (rc) return fail(rc, "elp_create: ncclCommInitAll failed");
        for (int r = 0; r < P; ++r) {
            HIPCHK(hipSetDevice(g->rank_dev[r]));
            rc = g->ranks[r]->comm.adopt_rccl(comms[r], P, r);
            if (rc) return fail(rc, "elp_create: communicator set-up failed");
        }
    } else {
        g->tgroup = std::make_unique<ThreadGroup>(P);
        g->tranks.resize(P);
        for (int r = 0; r < P; ++r) {
            g->tranks[r] = ThreadRank{g->tgroup.get(), r};
            g->ranks[r]->sel_cap = 32;  // (Dev::sel_cap: P - 1 spinning grids of <= 32 workgroups)
            HIPCHK(hipSetDevice(g->rank_dev[r]));
            const int rc = g->ranks[r]->comm.init_host(P, r, ThreadGroup::allgather, ThreadGroup::allreduce,
                                                       ThreadGroup::bcast, &g->tranks[r]);
            if (rc) return fail(rc, "elp_create: in-process transport set-up failed");
        }
    }
    g->peer_A.assign(P, nullptr);
    g->peer_A_bytes.assign(P, 0);
    enable_group_p2p(g);
    return 0;
}

extern "C" int elp_create(elp_handle** out, int64_t m, int64_t n, const elp_control* ctl) {
    if (!out) return fail(ELP_E_ARG, "elp_create: out is NULL");
    *out = nullptr;
    if (m < 0 || n < 1) return fail(ELP_E_ARG, "elp_create: need m >= 0 and n >= 1");
    if (m > 0x3fffffff || n > 0x3fffffff) return fail(ELP_E_ARG, "elp_create: dimension too large");
    if (ctl && ctl->pricing != ELP_PRICE_DANTZIG && ctl->pricing != ELP_PRICE_DEVEX)
        return fail(ELP_E_ARG, "elp_create: pricing must be ELP_PRICE_DANTZIG or ELP_PRICE_DEVEX");
    if (ctl && ctl->simplex != 0 && ctl->simplex != ELP_SIMPLEX_PRIMAL_PRIMAL && ctl->simplex != ELP_SIMPLEX_DUAL_PRIMAL)
        return fail(ELP_E_ARG, "elp_create: simplex must be 0, ELP_SIMPLEX_PRIMAL_PRIMAL or ELP_SIMPLEX_DUAL_PRIMAL");
    elp_handle* h = new elp_handle();
    if (ctl) h->ctl = *ctl;
    else elp_default_control(&h->ctl);
    if (h->ctl.refactor_period <= 0) h->ctl.refactor_period = 250;
    if (h->ctl.degen_switch <= 0) h->ctl.degen_switch = 50;
    if (h->ctl.sync_every <= 0) h->ctl.sync_every = 32;
    if (!(h->ctl.infinity > 0)) h->ctl.infinity = 1e30;
    if (!(h->ctl.tol_singular >= 0)) h->ctl.tol_singular = 1e-13;
    if (!(h->ctl.mailbox_timeout > 0)) h->ctl.mailbox_timeout = 2.0;
    if (h->ctl.ngpu < 1) h->ctl.ngpu = 1;
    h->m = m;
    h->n = n;
    h->col0 = 0;
    h->nloc = n;
    h->dev = h->ctl.device;
    if (hipSetDevice(h->dev) != hipSuccess) {
        delete h;
        return fail(ELP_E_HIP, "elp_create: hipSetDevice failed");
    }
    if (h->ctl.ngpu <= 1 && spares_on()) {
        std::lock_guard<std::mutex> lk(g_spare_mu);
        for (size_t i = g_spares.size(); i-- > 0;)
            if (g_spares[i].dev == h->dev) {
                Spare sp = std::move(g_spares[i]);
                g_spares.erase(g_spares.begin() + (long)i);
                h->st = sp.st;
                h->pool = std::move(sp.pool);
                h->keep_A = sp.keep_A;
                h->keep_A_bytes = sp.keep_A_bytes;
                h->hctl = sp.hctl;
                if (sp.resx_n == n) {  // (sized by n)
                    h->d_resout = sp.resout;
                    h->res_pin = sp.respin;
                } else {
                    if (sp.resout) (void)hipFree(sp.resout);
                    if (sp.respin) (void)hipHostFree(sp.respin);
                }
                break;
            }
    }
    if (!h->st && hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) {
        drain_pool(h);
        release_kept(h);
        delete h;
        return fail(ELP_E_HIP, "elp_create: stream creation failed");
    }
    if (h->ctl.ngpu > 1) {
        if (n < h->ctl.ngpu) {  // (prep_load's rule for column shards)
            elp_destroy(h);
            return fail(ELP_E_ARG, "elp_create: ngpu exceeds n (every rank prices at least one column)");
        }
        const int rc = create_group(h);
        if (rc) {
            const std::string msg = g_err;
            elp_destroy(h);
            return fail(rc, msg);
        }
    }
    *out = h;
    return 0;
}

// Allocate every device buffer for the local shard (called by elp_load_*).
static int alloc_all_body(elp_handle* h);
static int alloc_all(elp_handle* h) {
    t_alloc_h = h;
    const int rc = alloc_all_body(h);
    t_alloc_h = nullptr;
    drain_pool(h);  // what this shape did not take back
    return rc;
}
static int alloc_all_body(elp_handle* h) {
    Dev& d = h->d;
    const int64_t m = h->m, n = h->nloc;
    const int64_t mm = m > 0 ? m : 1;
    d.m = (int32_t)m;
    d.n = (int32_t)n;
    d.N = (int32_t)h->n;
    d.col0 = h->col0;
    d.world = h->comm.world;
    d.sharded = h->comm.kind != 0;
    d.nv = (int32_t)(n + 2 * m);
    // bump capacity: the explicit inverse needs O(m k + k^2), not O(m^2) -- k (the
    // basic structurals) starts at 0 and grows by at most one per iteration, so
    // the buffers start small and double at a poll (ensure_k)
    // a reload of the same shape starts at the capacities the last solve grew
    // to (the values never depend on them), so it does not grow again
    const bool same_shape = h->shape_m == m && h->shape_n == n && h->shape_csc == h->csc;
    const int64_t kcap_prev = same_shape ? h->kcap : 0, ar_prev = same_shape ? h->ar_rows : 0;
    h->shape_m = m;
    h->shape_n = n;
    h->shape_csc = h->csc;
    h->kcap = std::min<int64_t>(mm, std::max<int64_t>(256, kcap_prev));
    if (const char* e = std::getenv("ELP_KCAP_INIT"))  // test hook: force growth
        h->kcap = std::max<int64_t>(1, std::min<int64_t>(mm, std::atoll(e)));
    d.ldm = h->kcap;
    // pricing tiles (price_body): TILE_COLS columns each.  (r03 tried balanced
    // narrower tiles once there are 256+ -- every CU sweeping the same share:
    // slower at 5000 x 50000, 21.6 vs 19.9 us per launch, idle lanes and more
    // row loads cost more than the imbalance; removed in r06)
    d.tile_w = TILE_COLS;
    d.ntiles = (int32_t)std::max<int64_t>(1, (n + TILE_COLS - 1) / TILE_COLS);
    d.ldr = (int64_t)d.ntiles * d.tile_w;  // AR: [tile][row][tile_w], rows packed
    d.infinity = h->ctl.infinity;
    d.tol_singular = h->ctl.tol_singular;
    d.mb_ticks = (int64_t)(h->ctl.mailbox_timeout * 1e8);  // s_memrealtime: 100 MHz
    d.ptimer = ELP_DIAG && (h->ctl.verbose & ELP_PROFILE_PRICE) ? 1 : 0;  // (diagnostic builds)
    d.csc = h->csc ? 1 : 0;
    // CSC bumps above ELP_SPF_MIN (512) positions: sparse FTRAN and B^-1 rows
    // (DESIGN.md 9); below it the dense chains' prefetched rows win
    {
        static const int spf = [] {
            const char* s = std::getenv("ELP_SPF_MIN");
            return s ? std::atoi(s) : 512;
        }();
        d.spf_min = h->csc && spf > 0 ? spf : 0;
    }
    {  // one GPU: the dual phase's update deferred into the next iteration (A/B: ELP_DUAL_DEFER=0)
        static const bool dd = [] {
            const char* s = std::getenv("ELP_DUAL_DEFER");
            return !(s && std::atoi(s) == 0);
        }();
        d.dual_defer = dd && h->comm.kind == 0 ? 1 : 0;
    }
    {  // CSC: no MinvT (ELP_CSC_MINVT=1 keeps it, A/B)
        static const bool keep = [] {
            const char* s = std::getenv("ELP_CSC_MINVT");
            return s && std::atoi(s) != 0;
        }();
        d.noT = h->csc && !keep ? 1 : 0;
    }
    {  // CSC: the sparse rank-one inverse update (ELP_SRU=0: the dense one, A/B)
        static const bool off = [] {
            const char* s = std::getenv("ELP_SRU");
            return s && std::atoi(s) == 0;
        }();
        d.sru_on = h->csc && !off ? 1 : 0;
    }
    // the mailbox carries the min-loc record only: with A not replicated the
    // entering column must travel, so that load uses the collective
    d.p2p = h->comm.p2p && h->replicated ? 1 : 0;
    d.rank = h->comm.rank;
    d.mbox = (MboxRec*)h->comm.mbox;
    d.mpeers = (MboxRec* const*)h->comm.dpeers;
    d.force_select = std::getenv("ELP_FORCE_SELECT") ? 1 : 0;  // test hook
    d.sel_cap = h->sel_cap;
    const size_t nv = (size_t)(n + 2 * m);
    hipError_t e = hipSuccess;
    auto A = [&](hipError_t x) {
        if (e == hipSuccess) e = x;
    };
    // AR holds only the |Y| live rows: start small, grow at polls (ensure_ar)
    h->ar_rows = std::min<int64_t>(mm, std::max<int64_t>(1024, ar_prev));
    if (const char* e = std::getenv("ELP_AR_INIT_ROWS"))  // test hook: force growth
        h->ar_rows = std::max<int64_t>(1, std::min<int64_t>(mm, std::atoll(e)));
    if (h->csc) h->ar_rows = 1;  // CSC prices from the columns: no AR
    d.arcap = h->ar_rows;
    A(dalloc(&d.AR, (size_t)h->ar_rows * (size_t)d.ldr));
    // the explicit bump inverse's buffers (kcap positions, grown by ensure_k)
    const size_t msq = (size_t)h->kcap * (size_t)h->kcap;
    A(dalloc(&d.AS, (size_t)mm * (size_t)h->kcap));
    A(dalloc(&d.Minv, msq));
    if (!d.noT) A(dalloc(&d.MinvT, msq));
    A(dalloc(&d.cS, mm));
    A(dalloc(&d.slo, mm));
    A(dalloc(&d.shi, mm));
    A(dalloc(&d.rlo, mm));
    A(dalloc(&d.rhi, mm));
    A(dalloc(&d.b, mm));
    A(dalloc(&d.obj, n));
    A(dalloc(&d.lb, nv));
    A(dalloc(&d.ub, nv));
    A(dalloc(&d.cost, nv));
    A(dalloc(&d.xval, nv));
    A(dalloc(&d.vstat, nv));
    A(dalloc(&d.rowvs, mm));
    A(dalloc(&d.yvs, mm));
    A(dalloc(&d.dw, (size_t)(n + m)));
    A(dalloc(&d.dprev, (size_t)(n + m)));
    A(dalloc(&d.asgn, mm));
    A(dalloc(&d.xr, mm));
    A(dalloc(&d.xs, mm));
    A(dalloc(&d.y, mm));
    A(dalloc(&d.yy, mm));
    A(dalloc(&d.blockmin, (size_t)(mm / 32 + mm / 64 + 8)));  // k_ftran_zr row + bump tiles
    // pass-2 candidate regions: one per row tile (32 rows) and one per bump-tile
    // wave (64 positions): <= m/32 + k/64 + 8 (k <= m)
    d.rregs = (int32_t)(mm / 32 + mm / 64 + 10);
    A(dalloc(&d.rcand, (size_t)d.rregs * RREG));
    A(dalloc(&d.rcnt, (size_t)d.rregs));
    A(dalloc(&d.pkt, (size_t)(mm + 4)));
    A(dalloc(&d.objg, (size_t)h->n));
    A(dalloc(&d.ract, mm));
    A(dalloc(&d.cand_xchg, (size_t)h->comm.world));
    A(dalloc(&h->d_flag, 1));
    A(dalloc(&d.t, mm));
    A(dalloc(&d.acol, mm));
    A(dalloc(&d.aR, mm));
    A(dalloc(&d.alS, mm));
    A(dalloc(&d.alU, mm));
    A(dalloc(&d.zz, mm));
    A(dalloc(&d.zpart, (size_t)(mm + 64) * (size_t)((h->kcap + ZCHUNK - 1) / ZCHUNK + 1)));
    A(dalloc(&d.vrow, mm));
    A(dalloc(&d.vvec, mm));
    A(dalloc(&d.colA, mm));
    A(dalloc(&d.rhs, mm));
    A(dalloc(&d.cover, mm));
    A(dalloc(&d.rpos, mm));
    A(dalloc(&d.Rl, mm));
    A(dalloc(&d.Sl, mm));
    A(dalloc(&d.Yl, mm));
    A(dalloc(&d.ypos, mm));
    A(dalloc(&d.perm, mm));
    A(dalloc(&d.pivstep, mm));
    A(dalloc(&d.nzlist, n));
    A(dalloc(&d.nzchunk, n / (1024 * 16) + 2));
    A(dalloc(&d.nzcount, 1));
    // tile candidates + the slack workgroups' (|Y| <= m, >= 128 slots each)
    A(dalloc(&d.cand, (size_t)d.ntiles + (size_t)((mm + TILE_COLS - 1) / TILE_COLS) + 64));
    // one stamp pair per pricing workgroup: tiles, slack workgroups (<= m / 128 + 1)
    // and the apply workgroups (<= ELP_MINV_WG_MAX 8192 + 1024 copy workgroups,
    // launch_btran_price; the sparse update's <= 4096)
#ifdef ELP_PDBG
    A(dalloc(&d.pstamp, 6 * ((size_t)d.ntiles + (size_t)(mm / 128 + 1) + 8192 + 1024 + 64)));
#else
    A(dalloc(&d.pstamp, 2 * ((size_t)d.ntiles + (size_t)(mm / 128 + 1) + 8192 + 1024 + 64)));
#endif
    if (h->csc) A(dalloc(&d.qcol, mm));
    if (h->csc) A(dalloc(&d.spos, (size_t)(n > 0 ? n : 1)));  // (the sparse FTRAN-z's column -> position)
    if (!h->csc) A(dalloc(&d.qz, mm));  // (dense only)
    if (ELP_DIAG && std::getenv("ELP_STAMPS")) {  // (diagnostic builds)
        A(dalloc(&d.dstamp, DSTAMP_STRIDE * 64));
        d.stamp_wide = std::atoi(std::getenv("ELP_STAMPS")) >= 2;
    }
    // the release pricing timer's stamps (launch_btran_price's largest grid:
    // tiles + slack workgroups + deferred-update workgroups)
    d.ptslots = 64;
    d.ptcap = (int32_t)(d.ntiles + (mm / 128 + 1) + 8192 + 1024 + 64);
    A(dalloc(&d.ptst, 2 * (size_t)d.ptslots * (size_t)d.ptcap));
    A(dalloc(&d.ptgrid, (size_t)d.ptslots));
    A(dalloc(&d.ctl, 1));
    A(dalloc(&d.trace, (size_t)(h->trace_cap > 0 ? 2 * h->trace_cap : 2)));
    // dual simplex phase 1 (elp_kernels.hip "dual simplex"): regions = the
    // pricing tiles + the slack workgroups (<= m / 128 + 1), DREG slots each.
    // One GPU, or column-sharded ranks holding all of A (the flipped and the
    // entering columns are read from the replicated copy); the ratio test sees
    // every rank's candidates: up to N + m of them
    if (!d.sharded || !h->csc) {
        const int64_t Ng = h->n;
        d.dregs = d.ntiles + (int32_t)((mm + TILE_COLS - 1) / TILE_COLS) + 2;
        d.dchzn = (int32_t)((2 * mm + 255) / 256 + 2);
        A(dalloc(&d.rhoR, mm));
        A(dalloc(&d.rr, mm));
        A(dalloc(&d.dchz, (size_t)d.dchzn));
        A(dalloc(&d.dcand, (size_t)d.dregs * DREG));
        A(dalloc(&d.dcnt, (size_t)d.dregs));
        A(dalloc(&d.dcomp, (size_t)(Ng + m)));
        A(dalloc(&d.dalive, (size_t)(Ng + m)));
        A(dalloc(&d.dflip, (size_t)(Ng + m)));
        A(dalloc(&d.dflipdx, (size_t)(Ng + m)));
        A(dalloc(&d.aF, mm));
        A(dalloc(&d.fS, mm));
        if (h->csc) {  // (a_F's support and sparse a_F[R], k_dual_bfrt's tail)
            A(dalloc(&d.afs, (size_t)(1 + 1024)));
            A(dalloc(&d.afl, (size_t)(AFL_POS + 256)));
            A(dalloc(&d.aflv, (size_t)256));
            Fill32List fc{};  // -1: clear all of a_F first; -1: no list
            fc.f[0] = Fill32{d.afs, 1, 0xffffffffu, 0};
            fc.f[1] = Fill32{d.afl, 1, 0xffffffffu, 0};
            fc.count = 2;
            A(launch_fill32(fc, h->st));
        }
        d.dslack = !d.sharded || h->comm.rank == h->comm.world - 1;
        if (d.sharded) {
            const int P = h->comm.world;
            d.dcap = (int32_t)((Ng + P - 1) / P + m);  // a shard's columns (<= ceil(N / P)) + the slacks
            A(dalloc(&d.dsend, (size_t)d.dcap + 1));
            A(dalloc(&d.drecv, (size_t)P * ((size_t)d.dcap + 1)));
            A(dalloc(&d.ddw, (size_t)(Ng + 2 * m)));
        }
    }
    if (!d.ddw) d.ddw = d.dw;  // (one GPU: local ids are the global ids)
    A(dalloc(&h->ld_stage, (size_t)(2 * n + mm)));
    if (e != hipSuccess) {
        free_dev(h);
        return fail(ELP_E_NOMEM, std::string("device allocation failed: ") + hipGetErrorString(e));
    }
    if (!h->hctl) A(hipHostMalloc((void**)&h->hctl, sizeof(DevCtl)));
    // (AR padding columns [n, ldr) are read by the 128-column tiles but their
    //  results are discarded, so AR needs no clearing); Minv / work start clean
    // (one launch for all of them: a small LP's load is its launches)
    Fill32List fl{};
    auto fill = [&](void* p, int64_t words, uint32_t v) {
        if (p && fl.count < FILL32_MAX) fl.f[fl.count++] = Fill32{p, words, v, 0};
    };
    fill(d.rcnt, d.rregs, 0u);
    fill(d.Minv, 2 * (int64_t)msq, 0u);
    fill(d.MinvT, 2 * (int64_t)msq, 0u);
    fill(d.qcol, 2 * mm, 0u);
    // index lists: entries past k / |Y| are read speculatively (and discarded):
    // start them at -1 rather than whatever the allocator hands out
    for (int32_t* lst : {d.Rl, d.Sl, d.Yl, d.rpos, d.ypos}) fill(lst, mm, 0xffffffffu);
    A(launch_fill32(fl, h->st));

    if (e != hipSuccess) {
        free_dev(h);
        return fail(ELP_E_HIP, std::string("device init failed: ") + hipGetErrorString(e));
    }
    return 0;
}

// Grow AR to hold at least `rows` Y rows (device idle: called at a poll).
static int ensure_ar(elp_handle* h, int64_t rows) {
    if (h->csc) return 0;
    rows = std::min<int64_t>(rows, std::max<int64_t>(h->m, 1));
    if (rows <= h->ar_rows) return 0;
    const int64_t cap = std::min<int64_t>(std::max<int64_t>(h->m, 1), std::max(rows, 2 * h->ar_rows));
    double* nr = nullptr;
    if (hipMalloc((void**)&nr, (size_t)cap * (size_t)h->d.ldr * sizeof(double)) != hipSuccess)
        return fail(ELP_E_NOMEM, "AR growth failed");
    // tile-major layout: rows of each tile move to the new capacity
    double* old = h->d.AR;
    const int64_t old_cap = h->ar_rows;
    h->d.AR = nr;
    h->d.arcap = cap;
    h->ar_rows = cap;
    HIPCHK(hipMemcpyAsync(h->hctl, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    HIPCHK(launch_ar_relayout(h->d, old, old_cap, (int)std::min<int64_t>(old_cap, h->hctl->ny), h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    retire(h, old);
    return 0;
}

// Grow the bump buffers to hold at least `need` positions (device idle: called
// at a poll): AS keeps its first k columns (ld m), Minv / MinvT their k x k
// block (ld kcap -> the new kcap); zpart is scratch.
static int ensure_k(elp_handle* h, int64_t need) {
    const int64_t mm = std::max<int64_t>(h->m, 1);
    need = std::min<int64_t>(need, mm);
    if (need <= h->kcap) return 0;
    const int64_t cap = std::min<int64_t>(mm, std::max<int64_t>(need, 2 * h->kcap));
    HIPCHK(hipMemcpyAsync(h->hctl, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    const int64_t k = std::min<int64_t>(h->hctl->k + 1, h->kcap);  // (+1: a pending case-B plan's row)
    Dev& d = h->d;
    double *as = nullptr, *mi = nullptr, *mt = nullptr, *zp = nullptr;
    hipError_t e = dalloc(&as, (size_t)mm * (size_t)cap);
    if (e == hipSuccess) e = dalloc(&mi, (size_t)cap * (size_t)cap);
    if (e == hipSuccess && d.MinvT) e = dalloc(&mt, (size_t)cap * (size_t)cap);  // (none: CSC, d.noT)
    if (e == hipSuccess) e = dalloc(&zp, (size_t)(mm + 64) * (size_t)((cap + ZCHUNK - 1) / ZCHUNK + 1));
    if (e != hipSuccess) {
        for (double* p : {as, mi, mt, zp})
            if (p) (void)hipFree(p);
        return fail(ELP_E_NOMEM, "bump growth failed (k = " + std::to_string(need) + ")");
    }
    const size_t sq = (size_t)cap * (size_t)cap * sizeof(double);
    HIPCHK(hipMemsetAsync(mi, 0, sq, h->st));
    if (mt) HIPCHK(hipMemsetAsync(mt, 0, sq, h->st));
    if (k > 0) {
        HIPCHK(hipMemcpyAsync(as, d.AS, (size_t)k * (size_t)mm * sizeof(double), hipMemcpyDeviceToDevice, h->st));
        const size_t w = (size_t)k * sizeof(double);
        HIPCHK(hipMemcpy2DAsync(mi, (size_t)cap * sizeof(double), d.Minv, (size_t)h->kcap * sizeof(double), w,
                                (size_t)k, hipMemcpyDeviceToDevice, h->st));
        if (mt)
            HIPCHK(hipMemcpy2DAsync(mt, (size_t)cap * sizeof(double), d.MinvT, (size_t)h->kcap * sizeof(double), w,
                                    (size_t)k, hipMemcpyDeviceToDevice, h->st));
    }
    HIPCHK(hipStreamSynchronize(h->st));
    for (double* p : {d.AS, d.Minv, d.MinvT, d.zpart}) retire(h, p);
    d.AS = as;
    d.Minv = mi;
    d.MinvT = mt;
    d.zpart = zp;
    d.ldm = cap;
    h->kcap = cap;
    return 0;
}

static int ensure_w(elp_handle* h, int k) {
    const size_t need = (size_t)k * (size_t)k;
    if (need <= h->w_cap && h->d.W0) return 0;
    retire(h, h->d.W0);
    retire(h, h->d.W1);
    h->d.W0 = h->d.W1 = nullptr;
    size_t cap = std::max<size_t>(need, 64 * 64);
    cap = std::max(cap, h->w_cap * 2);
    if (dalloc(&h->d.W0, cap) != hipSuccess || dalloc(&h->d.W1, cap) != hipSuccess)
        return fail(ELP_E_NOMEM, "refactor workspace allocation failed");
    h->w_cap = cap;
    return 0;
}

// ract = sum_j a_ij x_j over nonzero nonbasic columns, in global column order:
// shard r continues the fma chain of shards 0..r-1 (broadcast after each turn)
static int row_chain(elp_handle* h) {
    const size_t mb = (size_t)h->m * sizeof(double);
    if (h->m == 0) return 0;
    HIPCHK(hipMemsetAsync(h->d.ract, 0, mb, h->st));
    if (h->comm.kind == 0) {
        HIPCHK(launch_row_chain(h->d, h->st));
        return 0;
    }
    for (int r = 0; r < h->comm.world; ++r) {
        if (r == h->comm.rank) HIPCHK(launch_row_chain(h->d, h->st));
        const int rc = h->comm.bcast_f64(h->d.ract, (size_t)h->m, r, h->st);
        if (rc) return fail(rc, "row activity broadcast failed");
    }
    return 0;
}

// max over ranks of an int decided on the host
static int any_rank(elp_handle* h, int v, int* out) {
    *out = v;
    if (h->comm.kind == 0) return 0;
    HIPCHK(hipMemcpyAsync(h->d_flag, &v, sizeof(int32_t), hipMemcpyHostToDevice, h->st));
    const int rc = h->comm.allreduce_max_i32(h->d_flag, 1, h->st);
    if (rc) return fail(rc, "flag all-reduce failed");
    int32_t r = 0;
    HIPCHK(hipMemcpyAsync(&r, h->d_flag, sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    *out = r;
    return 0;
}

// ELP_DEBUG_LOAD: phase times of elp_load_* on stderr (device synchronised)
static void load_mark(elp_handle* h, const char* what) {
    static const bool on = std::getenv("ELP_DEBUG_LOAD") != nullptr;
    if (!on) return;
    (void)hipStreamSynchronize(h->st);
    static thread_local double t_last = 0.0;
    const double t = now_s();
    if (what) std::fprintf(stderr, "elp load: %-18s %8.2f ms\n", what, 1e3 * (t - t_last));
    t_last = t;
}

static bool scaling_on(const elp_handle* h) { return (h->ctl.scaling & (ELP_SCALE_GEOMETRIC | ELP_SCALE_EQUILIBRATE)) != 0; }
static double unscale_col(const elp_handle* h, double v, int64_t j, int sgn) {
    return h->scol_h.empty() ? v : std::ldexp(v, sgn * h->scol_h[(size_t)j]);
}
static double unscale_row(const elp_handle* h, double v, int64_t i, int sgn) {
    return h->srow_h.empty() ? v : std::ldexp(v, sgn * h->srow_h[(size_t)i]);
}

// Scale the m x ncols column-major A in place on the device (launch_scale_*;
// oracle/elp_oracle.c scale_factors) and keep the exponents on the host.  A
// holds columns [c0, c0 + ncols): all N of them (one GPU, replicated shards:
// every rank computes the same factors alone), or this rank's shard only --
// then the row passes combine the shards' maxima with an all-reduce and the
// column exponents are gathered (exact f64 sum of a zero-filled vector).
static int scale_dense(elp_handle* h, double* A, int64_t c0, int64_t ncols, bool apply = true) {
    h->srow_h.clear();
    h->scol_h.clear();
    if (!scaling_on(h)) return 0;
    const int m = (int)h->m;
    const bool shards = ncols < h->n && h->comm.kind != 0;
    int32_t *rho = nullptr, *gam = nullptr, *rw = nullptr, *chg = nullptr;
    double* gg = nullptr;
    hipError_t e = dalloc(&rho, (size_t)std::max(m, 1));
    if (e == hipSuccess) e = dalloc(&gam, (size_t)std::max<int64_t>(ncols, 1));
    if (e == hipSuccess) e = dalloc(&rw, 2 * (size_t)std::max(m, 1));  // [rnm | rmx]
    if (e == hipSuccess) e = dalloc(&chg, 1);
    int32_t *rmn = rw, *rmx = rw + std::max(m, 1);
    if (e == hipSuccess) e = launch_scale_init(m, ncols, rho, gam, rmn, rmx, h->st);
    int rc = 0, passes = 0;
    const double t_sc = now_s();
    if (h->ctl.scaling & ELP_SCALE_GEOMETRIC)
        for (int pass = 0; pass < SCALE_PASSES && e == hipSuccess && !rc; ++pass) {
            passes++;
            int32_t moved = 0;
            e = hipMemsetAsync(chg, 0, sizeof(int32_t), h->st);
            if (e == hipSuccess) e = launch_scale_rows(m, ncols, A, gam, rmn, rmx, h->st);
            if (e == hipSuccess && shards) rc = h->comm.allreduce_max_i32(rw, 2 * (size_t)std::max(m, 1), h->st);
            if (e == hipSuccess && !rc) e = launch_scale_row_final(m, rmn, rmx, rho, chg, h->st);
            if (e == hipSuccess && !rc) e = launch_scale_cols(m, ncols, A, rho, gam, 0, chg, h->st);
            if (e == hipSuccess && !rc && shards) rc = h->comm.allreduce_max_i32(chg, 1, h->st);
            if (e == hipSuccess && !rc) e = hipMemcpyAsync(&moved, chg, sizeof(int32_t), hipMemcpyDeviceToHost, h->st);
            if (e == hipSuccess && !rc) e = hipStreamSynchronize(h->st);
            if (!moved) break;
        }
    if (e == hipSuccess && !rc && (h->ctl.scaling & ELP_SCALE_EQUILIBRATE))
        e = launch_scale_cols(m, ncols, A, rho, gam, 1, chg, h->st);
    if (e == hipSuccess && !rc && apply) e = launch_scale_apply(m, ncols, A, rho, gam, h->st);
    h->srow_h.assign((size_t)m, 0);
    h->scol_h.assign((size_t)h->n, 0);
    std::vector<int32_t> gl((size_t)ncols);
    if (e == hipSuccess && !rc && m)
        e = hipMemcpyAsync(h->srow_h.data(), rho, (size_t)m * sizeof(int32_t), hipMemcpyDeviceToHost, h->st);
    if (e == hipSuccess && !rc && ncols)
        e = hipMemcpyAsync(gl.data(), gam, (size_t)ncols * sizeof(int32_t), hipMemcpyDeviceToHost, h->st);
    if (e == hipSuccess && !rc) e = hipStreamSynchronize(h->st);
    if (e == hipSuccess && !rc) {
        if (!shards) {
            std::copy(gl.begin(), gl.end(), h->scol_h.begin() + c0);
        } else {  // every rank's column exponents
            std::vector<double> gv((size_t)h->n, 0.0);
            for (int64_t j = 0; j < ncols; ++j) gv[(size_t)(c0 + j)] = (double)gl[(size_t)j];
            e = dalloc(&gg, (size_t)h->n);
            if (e == hipSuccess)
                e = hipMemcpyAsync(gg, gv.data(), gv.size() * sizeof(double), hipMemcpyHostToDevice, h->st);
            if (e == hipSuccess) rc = h->comm.allreduce_sum_f64(gg, (size_t)h->n, h->st);
            if (e == hipSuccess && !rc)
                e = hipMemcpyAsync(gv.data(), gg, gv.size() * sizeof(double), hipMemcpyDeviceToHost, h->st);
            if (e == hipSuccess && !rc) e = hipStreamSynchronize(h->st);
            for (int64_t j = 0; j < h->n; ++j) h->scol_h[(size_t)j] = (int32_t)gv[(size_t)j];
        }
    }
    for (void* p : {(void*)rho, (void*)gam, (void*)rw, (void*)chg, (void*)gg})
        if (p) (void)hipFree(p);
    if (rc) return fail(rc, "scaling: shard exchange failed");
    if (e != hipSuccess) return fail(ELP_E_HIP, std::string("scaling: ") + hipGetErrorString(e));
    if (std::getenv("ELP_DEBUG_SCALE"))
        std::fprintf(stderr, "elp scaling: %d geometric passes, %.2f ms (m %lld, %lld columns)\n", passes,
                     1e3 * (now_s() - t_sc), (long long)m, (long long)ncols);
    return 0;
}

// The same factors from CSC arrays on the host (nonzeros only: explicit zeros
// are skipped exactly as the dense kernels skip zero entries); val is scaled in place.
static int ilogb_i(double a) { return std::ilogb(a); }
static int floor_half_h(int v) { return v >= 0 ? v / 2 : -((1 - v) / 2); }
static void scale_csc(elp_handle* h, const int64_t* cp, const int32_t* ri, double* val) {
    h->srow_h.clear();
    h->scol_h.clear();
    if (!scaling_on(h)) return;
    const int64_t m = h->m, n = h->n;
    constexpr int EMN = 0x3fffffff, EMX = -0x3fffffff;
    std::vector<int32_t> rho((size_t)m, 0), gam((size_t)n, 0);
    auto col_pass = [&](bool equil) {
        bool changed = false;
        for (int64_t j = 0; j < n; ++j) {
            int mn = EMN, mx = EMX;
            for (int64_t t = cp[j]; t < cp[j + 1]; ++t) {
                if (val[t] == 0.0) continue;  // (elp_load_csc rejects non-finite values)
                const int e = ilogb_i(val[t]) + rho[(size_t)ri[t]];
                mn = std::min(mn, e);
                mx = std::max(mx, e);
            }
            const int g = mx == EMX ? 0 : equil ? -(mx + 1) : -floor_half_h(mn + mx);
            if (g != gam[(size_t)j]) {
                gam[(size_t)j] = g;
                changed = true;
            }
        }
        return changed;
    };
    auto row_pass = [&]() {
        std::vector<int> mn((size_t)m, EMN), mx((size_t)m, EMX);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t t = cp[j]; t < cp[j + 1]; ++t) {
                if (val[t] == 0.0) continue;
                const int e = ilogb_i(val[t]) + gam[(size_t)j];
                const size_t i = (size_t)ri[t];
                mn[i] = std::min(mn[i], e);
                mx[i] = std::max(mx[i], e);
            }
        bool changed = false;
        for (int64_t i = 0; i < m; ++i) {
            const int r = mx[(size_t)i] == EMX ? 0 : -floor_half_h(mn[(size_t)i] + mx[(size_t)i]);
            if (r != rho[(size_t)i]) {
                rho[(size_t)i] = r;
                changed = true;
            }
        }
        return changed;
    };
    if (h->ctl.scaling & ELP_SCALE_GEOMETRIC)
        for (int pass = 0; pass < SCALE_PASSES; ++pass) {
            const bool ch = row_pass();
            if (!(col_pass(false) | ch)) break;
        }
    if (h->ctl.scaling & ELP_SCALE_EQUILIBRATE) col_pass(true);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t t = cp[j]; t < cp[j + 1]; ++t) val[t] = std::ldexp(val[t], rho[(size_t)ri[t]] + gam[(size_t)j]);
    h->srow_h = std::move(rho);
    h->scol_h = std::move(gam);
}

// The same factors for a small dense A on the host (m n <= SCALE_HOST_MAX:
// below that the device passes' launches and one synchronisation per pass cost
// more than the arithmetic -- 0.2 ms of a 0.4 ms load at the DOP LP's 11 x 14):
// the exponents of the nonzero finite entries once, then the passes of
// scale_dense's kernels on them; returns the scaled copy of A.
constexpr double SCALE_HOST_MAX = 16384.0;
static std::vector<double> scale_dense_host(elp_handle* h, const double* A) {
    const int64_t m = h->m, n = h->n;
    constexpr int EMN = 0x3fffffff, EMX = -0x3fffffff, NONE = INT32_MIN;
    std::vector<int32_t> ex((size_t)(m * n));
    for (int64_t t = 0; t < m * n; ++t)
        ex[(size_t)t] = (A[t] != 0.0 && std::isfinite(A[t])) ? ilogb_i(A[t]) : NONE;
    std::vector<int32_t> rho((size_t)m, 0), gam((size_t)n, 0);
    auto col_pass = [&](bool equil) {
        bool changed = false;
        for (int64_t j = 0; j < n; ++j) {
            int mn = EMN, mx = EMX;
            for (int64_t i = 0; i < m; ++i) {
                const int e0 = ex[(size_t)(j * m + i)];
                if (e0 == NONE) continue;
                const int e = e0 + rho[(size_t)i];
                mn = std::min(mn, e);
                mx = std::max(mx, e);
            }
            const int g = mx == EMX ? 0 : equil ? -(mx + 1) : -floor_half_h(mn + mx);
            if (g != gam[(size_t)j]) {
                gam[(size_t)j] = g;
                changed = true;
            }
        }
        return changed;
    };
    auto row_pass = [&]() {
        bool changed = false;
        for (int64_t i = 0; i < m; ++i) {
            int mn = EMN, mx = EMX;
            for (int64_t j = 0; j < n; ++j) {
                const int e0 = ex[(size_t)(j * m + i)];
                if (e0 == NONE) continue;
                const int e = e0 + gam[(size_t)j];
                mn = std::min(mn, e);
                mx = std::max(mx, e);
            }
            const int r = mx == EMX ? 0 : -floor_half_h(mn + mx);
            if (r != rho[(size_t)i]) {
                rho[(size_t)i] = r;
                changed = true;
            }
        }
        return changed;
    };
    if (h->ctl.scaling & ELP_SCALE_GEOMETRIC)
        for (int pass = 0; pass < SCALE_PASSES; ++pass) {
            const bool ch = row_pass();
            if (!(col_pass(false) | ch)) break;
        }
    if (h->ctl.scaling & ELP_SCALE_EQUILIBRATE) col_pass(true);
    std::vector<double> As((size_t)(m * n));
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < m; ++i)
            As[(size_t)(j * m + i)] = std::ldexp(A[j * m + i], rho[(size_t)i] + gam[(size_t)j]);
    h->srow_h = std::move(rho);
    h->scol_h = std::move(gam);
    return As;
}

// the phase-1 method (elp_control.simplex; lp_solve's set_simplextype): the
// dual simplex with the bump inverse, on one GPU or column-sharded
// (elp_stats.simplex reports what ran)
static int simplex_type(const elp_handle* h) {
    return h->ctl.simplex == 0 ? ELP_SIMPLEX_DEFAULT : h->ctl.simplex;
}
static bool dual_phase1(const elp_handle* h) {
    return simplex_type(h) == ELP_SIMPLEX_DUAL_PRIMAL && h->d.dcand &&
           (h->comm.kind == 0 || (!h->csc && h->d.dsend));
}

// common tail of elp_load_*: bounds, rows, control block, phase decision
static int load_common(elp_handle* h, const int32_t* dir, const double* rhs, const double* obj,
                       const double* lo, const double* up, int32_t maximize) {
    const int64_t m = h->m, n = h->n, n0 = h->col0, nl = h->nloc;
    Dev& d = h->d;
    h->res_fresh = false;
    h->res_warm = 0;
    h->ctl_fresh = false;
    load_mark(h, "A + scaling");
    for (int64_t i = 0; i < m; ++i)
        if (dir[i] < ELP_LE || dir[i] > ELP_EQ) return fail(ELP_E_ARG, "dir must be 1 (<=), 2 (>=) or 3 (==)");
    h->maximize = maximize ? 1 : 0;
    d.maximize = h->maximize;
    h->obj_h.assign(obj, obj + n);
    h->dir_h.assign(dir, dir + m);
    h->rhs_h.assign(rhs, rhs + m);
    if (!h->in_bnb) {  // a fresh problem: root bounds, no integer columns yet
        h->lo_h.assign(n, 0.0);
        h->up_h.assign(n, HUGE_VAL);
        for (int64_t j = 0; j < n; ++j) {
            if (lo) h->lo_h[j] = lo[j];
            if (up) h->up_h[j] = up[j];
        }
        h->is_int.clear();
        h->mip = false;
    }
    // host-side staging of the small vectors (local column shard), scaled:
    // bounds by 2^-scol, costs by 2^scol, rhs by 2^srow (infinite values first
    // become +-inf, so they stay infinite)
    const double BIG = h->ctl.infinity;
    auto fin = [&](double v) { return v <= -BIG ? -HUGE_VAL : v >= BIG ? HUGE_VAL : v; };
    std::vector<double> lo_h(nl), up_h(nl), slb(m), sub(m), rhs_s(m), obj_s(n);
    for (int64_t j = 0; j < nl; ++j) {
        lo_h[j] = unscale_col(h, fin(lo ? lo[n0 + j] : 0.0), n0 + j, -1);
        up_h[j] = unscale_col(h, fin(up ? up[n0 + j] : HUGE_VAL), n0 + j, -1);
    }
    for (int64_t i = 0; i < m; ++i) rhs_s[i] = unscale_row(h, fin(rhs[i]), i, 1);
    for (int64_t j = 0; j < n; ++j) obj_s[j] = unscale_col(h, obj[j], j, 1);
    for (int64_t i = 0; i < m; ++i) {
        slb[i] = dir[i] == ELP_GE ? -HUGE_VAL : 0.0;
        sub[i] = dir[i] == ELP_LE ? HUGE_VAL : 0.0;
    }
    double *dlo = h->ld_stage, *dup = h->ld_stage + nl, *drhs = h->ld_stage + 2 * nl;
    HIPCHK(hipMemcpyAsync(dlo, lo_h.data(), nl * sizeof(double), hipMemcpyHostToDevice, h->st));
    HIPCHK(hipMemcpyAsync(dup, up_h.data(), nl * sizeof(double), hipMemcpyHostToDevice, h->st));
    if (m) {
        HIPCHK(hipMemcpyAsync(drhs, rhs_s.data(), m * sizeof(double), hipMemcpyHostToDevice, h->st));
        HIPCHK(hipMemcpyAsync(d.lb + nl, slb.data(), m * sizeof(double), hipMemcpyHostToDevice, h->st));
        HIPCHK(hipMemcpyAsync(d.ub + nl, sub.data(), m * sizeof(double), hipMemcpyHostToDevice, h->st));
    }
    HIPCHK(hipMemcpyAsync(d.obj, obj_s.data() + n0, nl * sizeof(double), hipMemcpyHostToDevice, h->st));
    HIPCHK(hipMemcpyAsync(d.objg, obj_s.data(), n * sizeof(double), hipMemcpyHostToDevice, h->st));
    DevCtl c{};
    c.status = ST_RUN;
    c.phase = 1;
    c.iter_limit = h->ctl.max_iter > 0 ? h->ctl.max_iter : 100 * (m + n) + 10000;
    // branch and bound: max_iter bounds the whole tree, not each node
    if (h->in_bnb && h->ctl.max_iter > 0) c.iter_limit = std::max<int64_t>(h->bnb_iter_left, 0);
    c.iter_stop = INT64_MAX;
    c.refactor_period = h->ctl.refactor_period;
    c.degen_switch = h->ctl.degen_switch;
    c.tol_primal = h->ctl.tol_primal;
    c.tol_dual = h->ctl.tol_dual;
    c.tol_pivot = h->ctl.tol_pivot;
    c.trace_cap = h->trace_cap;
    c.unb_var = -1;
    c.qcol_var = -1;
    c.mb_epoch = ++h->mb_epoch;
    c.devex = h->ctl.pricing == ELP_PRICE_DEVEX;
    c.dv_lv = -1;
    *h->hctl = c;
    HIPCHK(hipMemcpyAsync(d.ctl, h->hctl, sizeof(DevCtl), hipMemcpyHostToDevice, h->st));
    if (d.qcol) HIPCHK(hipMemsetAsync(d.qcol, 0, (size_t)std::max<int64_t>(m, 1) * sizeof(double), h->st));
    HIPCHK(launch_init_cols(d, dlo, dup, h->st));
    {
        const int rc = row_chain(h);
        if (rc) return rc;
    }
    HIPCHK(launch_init_rows(d, drhs, h->st));
    HIPCHK(launch_devex_reset(d, h->st));
    HIPCHK(hipMemcpyAsync(h->hctl, d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    {
        const int rc = ensure_ar(h, (int64_t)h->hctl->ny + 64);
        if (rc) return rc;
    }
    load_mark(h, "cols / rows / Y");
    // (r01-r05 kept an opt-in row-major copy of A for the AR row copies; with
    // and without it C3 and C4 measured the same and it doubled A's footprint:
    // removed in r06 -- the copies read A's rows in place)
    release_kept(h);  // whatever this load did not take
    HIPCHK(launch_fill_AR(h->d, h->st));
    int infeasible = 0;
    {
        const int rc = any_rank(h, h->hctl->infeasible_bounds, &infeasible);
        if (rc) return rc;
    }
    h->k_sync = 0;
    h->ny_sync = h->hctl->ny;
    h->since_refactor_sync = 0;
    h->any_art = h->hctl->ny > 0;
    h->loaded = true;
    h->done = false;
    h->stats = elp_stats{};
    h->stats.world_size = h->comm.world;
    h->stats.rank = h->comm.rank;
    h->stats.col0 = h->col0;
    h->stats.ncols = h->nloc;
    h->stats.exchange = h->comm.kind == 0 ? 0 : d.p2p ? 1 : 2;
    h->stats.basis = ELP_BASIS_INVERSE;
    h->timing_started = false;
    if (infeasible) {  // R/class.R:297-298: lower > upper -> "unfeasible"
        h->done = true;
        h->final_status = ELP_INFEASIBLE;
        return 0;
    }
    h->dual_used = false;
    if (h->any_art && dual_phase1(h)) {
        // SIMPLEX_DUAL_PRIMAL (oracle solve_core): the slack basis is infeasible,
        // so the phase-1 method is the dual simplex from a dual-feasible start --
        // boxed columns at the bound their cost sign asks for, the costs no bound
        // makes dual feasible zeroed, every row covered by its slack
        HIPCHK(launch_dual_setup_cols(d, h->st));
        {
            const int rc = row_chain(h);
            if (rc) return rc;
        }
        HIPCHK(launch_dual_init_rows(d, h->st));
        HIPCHK(launch_btran_exact(d, 0, h->st));  // slack basis: y = 0
        HIPCHK(hipMemcpyAsync(h->hctl, d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
        HIPCHK(hipStreamSynchronize(h->st));
        h->hctl->phase = 2;
        h->hctl->devex = 0;  // (the primal Devex weights: dw holds the dual ones)
        h->hctl->ddevex = h->ctl.pricing == ELP_PRICE_DEVEX;
        HIPCHK(hipMemcpyAsync(d.ctl, h->hctl, sizeof(DevCtl), hipMemcpyHostToDevice, h->st));
        h->phase = 3;
        h->any_art = false;
        h->dual_used = true;
        h->ctl_fresh = true;  // (no wait: the stream orders what reads it)
    } else if (h->any_art) {
        h->phase = 1;
    } else {
        HIPCHK(launch_phase2(d, h->st));
        h->phase = 2;
        HIPCHK(launch_btran_exact(d, 0, h->st));  // slack basis: y = 0
        c = *h->hctl;
        h->hctl->phase = 2;
        HIPCHK(hipMemcpyAsync(&d.ctl->phase, &h->hctl->phase, sizeof(int32_t), hipMemcpyHostToDevice, h->st));
        HIPCHK(hipStreamSynchronize(h->st));
    }
    return 0;
}

// ---------------------------------------------------------------- host -> device
// elp_load_dense's copy of A from the caller's pageable memory (the R matrix,
// the one H2D copy that replaces the add.constraint loop).  A
// pageable hipMemcpy stages through the runtime's own small pinned buffers one
// at a time; here host threads copy chunk c into pinned buffer c % STAGE_BUFS
// while the DMA engines move the chunks before it, and every device that needs
// a range of A (all ranks of an ngpu handle) receives each chunk from the same
// pinned buffer -- A is read from host memory once however many devices get it.
namespace {
constexpr size_t STAGE_BYTES = (size_t)16 << 20;  // per chunk
constexpr int STAGE_BUFS = 6;
constexpr size_t STAGE_MIN = (size_t)8 << 20;     // below this: one plain copy

struct H2DTarget {
    int dev;
    hipStream_t st;
    double* dst;    // receives source elements [e0, e1)
    size_t e0, e1;
};

// persistent pinned chunks (process lifetime: pinning 96 MB costs more than
// most loads); one staged upload at a time
std::mutex g_stage_mu;
void* g_stage[STAGE_BUFS] = {};

// memcpy of one chunk split over T host threads (memory-bandwidth bound: one
// thread reaches ~1/4 of what the DMA engines take)
struct CopyPool {
    int T;
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv, done;
    const char* src = nullptr;
    char* dst = nullptr;
    size_t bytes = 0;
    uint64_t gen = 0;
    int pending = 0;
    bool quit = false;
    explicit CopyPool(int t) : T(t) {
        for (int i = 0; i < T; ++i) th.emplace_back([this, i] { work(i); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
    }
    void work(int i) {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return quit || gen != seen; });
            if (quit) return;
            seen = gen;
            const char* s = src;
            char* d = dst;
            const size_t b = bytes;
            lk.unlock();
            size_t per = (b + (size_t)T - 1) / (size_t)T;
            per = (per + 4095) & ~(size_t)4095;
            const size_t o = (size_t)i * per;
            if (o < b) std::memcpy(d + o, s + o, std::min(per, b - o));
            lk.lock();
            if (--pending == 0) done.notify_one();
        }
    }
    void copy(void* d, const void* s, size_t b) {
        {
            std::lock_guard<std::mutex> lk(mu);
            src = static_cast<const char*>(s);
            dst = static_cast<char*>(d);
            bytes = b;
            pending = T;
            ++gen;
        }
        cv.notify_all();
        std::unique_lock<std::mutex> lk(mu);
        done.wait(lk, [&] { return pending == 0; });
    }
};
}  // namespace

// copy src[e0, e1) of every target to its device; returns after every DMA is done
static int h2d_staged(const double* src, std::vector<H2DTarget>& tg) {
    size_t lo = SIZE_MAX, hi = 0;
    for (const H2DTarget& t : tg)
        if (t.e1 > t.e0) {
            lo = std::min(lo, t.e0);
            hi = std::max(hi, t.e1);
        }
    if (hi <= lo) return 0;
    if ((hi - lo) * sizeof(double) < STAGE_MIN) {
        // (a pageable source is consumed before the call returns; one device's
        //  stream orders the rest of the load behind the copy: no wait)
        for (const H2DTarget& t : tg)
            if (t.e1 > t.e0) {
                HIPCHK(hipSetDevice(t.dev));
                HIPCHK(hipMemcpyAsync(t.dst, src + t.e0, (t.e1 - t.e0) * sizeof(double), hipMemcpyHostToDevice,
                                      t.st));
                if (tg.size() > 1) HIPCHK(hipStreamSynchronize(t.st));
            }
        return 0;
    }
    std::lock_guard<std::mutex> lk(g_stage_mu);
    for (int b = 0; b < STAGE_BUFS; ++b)
        if (!g_stage[b] && hipHostMalloc(&g_stage[b], STAGE_BYTES, hipHostMallocDefault) != hipSuccess) {
            g_stage[b] = nullptr;
            return fail(ELP_E_NOMEM, "elp_load_dense: pinned staging allocation failed");
        }
    const size_t P = tg.size();
    std::vector<hipEvent_t> ev(P * STAGE_BUFS, nullptr);
    std::vector<char> used(P * STAGE_BUFS, 0);
    int rc = 0;
    for (size_t t = 0; t < P && !rc; ++t)
        for (int b = 0; b < STAGE_BUFS && !rc; ++b)
            if (hipSetDevice(tg[t].dev) != hipSuccess ||
                hipEventCreateWithFlags(&ev[t * STAGE_BUFS + b], hipEventDisableTiming) != hipSuccess)
                rc = fail(ELP_E_HIP, "elp_load_dense: event creation failed");
    if (!rc) {
        const unsigned hw = std::thread::hardware_concurrency();
        CopyPool pool((int)std::max(1u, std::min(8u, hw ? hw : 1u)));
        const size_t ce = STAGE_BYTES / sizeof(double);
        size_t c = 0;
        for (size_t e = lo; e < hi && !rc; e += ce, ++c) {
            const size_t f = std::min(hi, e + ce);
            const int b = (int)(c % STAGE_BUFS);
            for (size_t t = 0; t < P && !rc; ++t)  // buffer b's last DMAs are done
                if (used[t * STAGE_BUFS + b] && hipEventSynchronize(ev[t * STAGE_BUFS + b]) != hipSuccess)
                    rc = fail(ELP_E_HIP, "elp_load_dense: staging wait failed");
            if (rc) break;
            pool.copy(g_stage[b], src + e, (f - e) * sizeof(double));
            for (size_t t = 0; t < P && !rc; ++t) {
                const size_t a0 = std::max(e, tg[t].e0), a1 = std::min(f, tg[t].e1);
                if (a1 <= a0) continue;
                if (hipSetDevice(tg[t].dev) != hipSuccess ||
                    hipMemcpyAsync(tg[t].dst + (a0 - tg[t].e0), static_cast<double*>(g_stage[b]) + (a0 - e),
                                   (a1 - a0) * sizeof(double), hipMemcpyHostToDevice, tg[t].st) != hipSuccess ||
                    hipEventRecord(ev[t * STAGE_BUFS + b], tg[t].st) != hipSuccess)
                    rc = fail(ELP_E_HIP, "elp_load_dense: staged copy failed");
                used[t * STAGE_BUFS + b] = 1;
            }
        }
    }
    for (size_t t = 0; t < P; ++t) {
        (void)hipSetDevice(tg[t].dev);
        if (hipStreamSynchronize(tg[t].st) != hipSuccess && !rc) rc = fail(ELP_E_HIP, "elp_load_dense: H2D failed");
        for (int b = 0; b < STAGE_BUFS; ++b)
            if (ev[t * STAGE_BUFS + b]) (void)hipEventDestroy(ev[t * STAGE_BUFS + b]);
    }
    return rc;
}

// will this rank hold all of A (prep_load's rule, before prep_load ran)?
static bool will_replicate(const elp_handle* h) {
    const double abytes = 8.0 * (double)h->m * (double)h->n;
    return h->comm.kind != 0 && (h->ctl.replicate == 1 || (h->ctl.replicate == 0 && abytes <= 64.0 * (1ull << 30)));
}
static int64_t shard_col0(const elp_handle* h) {
    return h->comm.world > 1 ? (int64_t)h->comm.rank * h->n / h->comm.world : 0;
}
static int64_t shard_ncols(const elp_handle* h) {
    if (h->comm.world <= 1) return h->n;
    const int64_t P = h->comm.world, r = h->comm.rank;
    return (r + 1) * h->n / P - r * h->n / P;
}

static int prep_load(elp_handle* h, bool csc = false) {
    if (!h) return fail(ELP_E_ARG, "NULL handle");
    HIPCHK(hipSetDevice(h->dev));
    h->res_fresh = false;
    h->res_warm = 0;
    h->ctl_fresh = false;
    load_mark(h, nullptr);
    if (h->loaded) free_dev(h, true);
    load_mark(h, "free previous");
    h->loaded = false;
    h->csc = csc;
    if (h->ctl.basis == ELP_BASIS_LU)  // (the r03-r04 sparse-LU engine, removed in r05: DESIGN.md 9.1)
        return fail(ELP_E_UNSUPPORTED, "elp_control.basis = ELP_BASIS_LU: the sparse-LU engine was removed "
                                       "(150x slower than the bump inverse); use ELP_BASIS_AUTO / _INVERSE");
    if (csc && h->comm.kind != 0)
        return fail(ELP_E_UNSUPPORTED, "elp_load_csc: column-sharded CSC solves are not supported");
    if (h->comm.world > 1) {
        const int64_t P = h->comm.world, r = h->comm.rank;
        if (h->n < P)  // every rank prices at least one column
            return fail(ELP_E_ARG, "column-sharded solve: n (" + std::to_string(h->n) + ") is below the rank count (" +
                                       std::to_string(P) + ")");
        h->col0 = r * h->n / P;
        h->nloc = (r + 1) * h->n / P - h->col0;
    }
    // replicate A on every rank when it fits (288 GB of HBM per MI355X): the
    // entering column is then read locally and never exchanged
    const double abytes = 8.0 * (double)h->m * (double)h->n;
    h->replicated = h->comm.kind != 0 &&
                    (h->ctl.replicate == 1 || (h->ctl.replicate == 0 && abytes <= 64.0 * (1ull << 30)));
    const int rc = alloc_all(h);
    load_mark(h, "alloc");
    return rc;
}

// elp_load_dense, part 1: the device copy of A this rank owns (all of A when
// replicated, else its column shard), allocated but not yet filled
static int dense_host_prepare(elp_handle* h) {
    int rc = prep_load(h);
    if (rc) return rc;
    const int64_t nc = h->replicated ? h->n : h->nloc;
    const size_t cnt = (size_t)h->m * (size_t)nc;
    HIPCHK(take_or_alloc(&h->A_owned, cnt * sizeof(double), &h->keep_A, &h->keep_A_bytes));
    h->A_owned_bytes = cnt * sizeof(double);
    return 0;
}
// the source range [e0, e1) of the column-major host A this rank receives
static H2DTarget dense_host_target(elp_handle* h) {
    const int64_t c0 = h->replicated ? 0 : h->col0, nc = h->replicated ? h->n : h->nloc;
    return H2DTarget{h->dev, h->st, h->A_owned, (size_t)c0 * (size_t)h->m, (size_t)(c0 + nc) * (size_t)h->m};
}
// part 2 (A uploaded): scaling in place, then the common tail
static int dense_host_finish(elp_handle* h, const int32_t* dir, const double* rhs, const double* obj,
                             const double* lo, const double* up, int32_t maximize, bool host_scaled = false) {
    HIPCHK(hipSetDevice(h->dev));
    const int64_t c0 = h->replicated ? 0 : h->col0, nc = h->replicated ? h->n : h->nloc;
    if (!host_scaled) {
        const int rc = scale_dense(h, h->A_owned, c0, nc);
        if (rc) return rc;
    }
    h->d.A = h->A_owned + (size_t)(h->col0 - c0) * (size_t)h->m;
    h->d.Afull = h->replicated ? h->A_owned : nullptr;
    return load_common(h, dir, rhs, obj, lo, up, maximize);
}

extern "C" int elp_load_dense(elp_handle* h, const double* A, const int32_t* dir, const double* rhs,
                              const double* obj, const double* lo, const double* up, int32_t maximize) {
    const double t0 = now_s();
    if (!h || !obj || (h->m > 0 && (!A || !dir || !rhs))) return fail(ELP_E_ARG, "elp_load_dense: NULL input");
    std::vector<elp_handle*> rk;
    if (is_group(h)) {
        rk = h->ranks;
        int rc = fan_out(h, [&](elp_handle* r, int) { return dense_host_prepare(r); });
        if (rc) return rc;
    } else {
        rk.push_back(h);
        int rc = dense_host_prepare(h);
        if (rc) return rc;
    }
    // A crosses PCIe once per device that needs it, from one pass over host memory
    std::vector<H2DTarget> tg;
    double hbytes = 0.0;
    size_t lo_e = SIZE_MAX, hi_e = 0;
    for (elp_handle* r : rk) {
        tg.push_back(dense_host_target(r));
        lo_e = std::min(lo_e, tg.back().e0);
        hi_e = std::max(hi_e, tg.back().e1);
    }
    if (hi_e > lo_e) hbytes = (double)(hi_e - lo_e) * sizeof(double);
    // a small A on one GPU is scaled on the host and crosses scaled
    const bool host_scale = !is_group(h) && h->comm.kind == 0 && scaling_on(h) && h->m > 0 &&
                            (double)h->m * (double)h->n <= SCALE_HOST_MAX;
    std::vector<double> As;
    if (host_scale) As = scale_dense_host(h, A);
    const double t1 = now_s();
    int rc = h2d_staged(host_scale ? As.data() : A, tg);
    const double th2d = now_s() - t1;
    if (rc) return rc;
    if (is_group(h))
        rc = fan_out(h, [&](elp_handle* r, int) { return dense_host_finish(r, dir, rhs, obj, lo, up, maximize); });
    else
        rc = dense_host_finish(h, dir, rhs, obj, lo, up, maximize, host_scale);
    for (elp_handle* r : rk) {
        r->stats.seconds_load = now_s() - t0;
        r->stats.seconds_h2d = th2d;
        r->stats.h2d_bytes = hbytes;
    }
    return rc;
}

extern "C" int elp_load_dense_device(elp_handle* h, const double* dA, const int32_t* dir,
                                     const double* rhs, const double* obj, const double* lo,
                                     const double* up, int32_t maximize) {
    if (is_group(h)) {
        // every rank reads A from its own HBM: ranks on other devices get a copy
        // of what they read -- all of A when replicated, else their column shard
        // (addressed through the full-shape base, so d.A = base + col0 * m)
        return fan_out(h, [&](elp_handle* r, int k) {
            const double* src = dA;
            const int64_t c0 = will_replicate(r) ? 0 : shard_col0(r);
            const int64_t nc = will_replicate(r) ? r->n : shard_ncols(r);
            const size_t cnt = (size_t)h->m * (size_t)nc;
            if (cnt && h->rank_dev[k] != h->rank_dev[0]) {
                if (hipSetDevice(h->rank_dev[k]) != hipSuccess) return fail(ELP_E_HIP, "hipSetDevice");
                if (!h->peer_A[k] || h->peer_A_bytes[k] != cnt) {
                    if (h->peer_A[k]) (void)hipFree(h->peer_A[k]);
                    h->peer_A[k] = nullptr;
                    h->peer_A_bytes[k] = 0;
                    if (dalloc(&h->peer_A[k], cnt) != hipSuccess) return fail(ELP_E_NOMEM, "copy of A");
                    h->peer_A_bytes[k] = cnt;
                }
                if (hipMemcpyPeer(h->peer_A[k], h->rank_dev[k], dA + (size_t)c0 * (size_t)h->m, h->rank_dev[0],
                                  cnt * sizeof(double)) != hipSuccess)
                    return fail(ELP_E_HIP, "hipMemcpyPeer of A");
                src = h->peer_A[k] - (size_t)c0 * (size_t)h->m;
            }
            return elp_load_dense_device(r, src, dir, rhs, obj, lo, up, maximize);
        });
    }
    const double t0 = now_s();
    if (!h || !obj || (h->m > 0 && (!dA || !dir || !rhs)))
        return fail(ELP_E_ARG, "elp_load_dense_device: NULL input");
    int rc = prep_load(h);
    if (rc) return rc;
    if (scaling_on(h)) {
        // the caller's A is read-only and may be large (40 GB at 10 000 x 500 000):
        // the factors come from read-only passes and every kernel scales what it
        // reads on the fly (Dev::srow / scol; exact, the values of a scaled copy)
        const int64_t c0 = h->replicated ? 0 : h->col0, nc = h->replicated ? h->n : h->nloc;
        rc = scale_dense(h, const_cast<double*>(dA) + (size_t)c0 * (size_t)h->m, c0, nc, false);
        if (rc) return rc;
        int32_t *sr = nullptr, *scg = nullptr;
        HIPCHK(dalloc(&sr, (size_t)std::max<int64_t>(h->m, 1)));
        HIPCHK(dalloc(&scg, (size_t)h->n));
        h->d.srow = sr;
        h->d.scol = scg;
        if (h->m)
            HIPCHK(hipMemcpyAsync(sr, h->srow_h.data(), (size_t)h->m * sizeof(int32_t), hipMemcpyHostToDevice, h->st));
        HIPCHK(hipMemcpyAsync(scg, h->scol_h.data(), (size_t)h->n * sizeof(int32_t), hipMemcpyHostToDevice, h->st));
    } else {
        h->srow_h.clear();
        h->scol_h.clear();
    }
    h->d.A = dA + (size_t)h->col0 * (size_t)h->m;
    h->d.Afull = h->replicated ? dA : nullptr;
    rc = load_common(h, dir, rhs, obj, lo, up, maximize);
    h->stats.seconds_load = now_s() - t0;
    return rc;
}

extern "C" int elp_load_dense_device_multi(elp_handle* h, const double* const* dA, int32_t count,
                                           const int32_t* dir, const double* rhs, const double* obj,
                                           const double* lo, const double* up, int32_t maximize) {
    if (!h || !dA) return fail(ELP_E_ARG, "elp_load_dense_device_multi: NULL argument");
    const int P = is_group(h) ? (int)h->ranks.size() : 1;
    if (count != P)
        return fail(ELP_E_ARG, "elp_load_dense_device_multi: count must equal the handle's rank count (" +
                                   std::to_string(P) + ")");
    if (!is_group(h)) return elp_load_dense_device(h, dA[0], dir, rhs, obj, lo, up, maximize);
    return fan_out(h, [&](elp_handle* r, int k) { return elp_load_dense_device(r, dA[k], dir, rhs, obj, lo, up, maximize); });
}

// CSC input: validate, build the CSR copy on the host (row activities), upload.
extern "C" int elp_load_csc(elp_handle* h, const int64_t* colptr, const int32_t* rowind,
                            const double* val, const int32_t* dir, const double* rhs,
                            const double* obj, const double* lo, const double* up, int32_t maximize) {
    if (is_group(h)) return fail(ELP_E_UNSUPPORTED, "elp_load_csc: not with ngpu > 1 (column-sharded CSC)");
    const double t0 = now_s();
    if (!h || !obj || !colptr || (h->m > 0 && (!dir || !rhs))) return fail(ELP_E_ARG, "elp_load_csc: NULL input");
    const int64_t m = h->m, n = h->n;
    const int64_t nnz = colptr[n];
    if (colptr[0] != 0 || nnz < 0 || (nnz > 0 && (!rowind || !val)))
        return fail(ELP_E_ARG, "elp_load_csc: colptr[0] must be 0 and colptr[n] = nnz >= 0");
    if (nnz > INT32_MAX) return fail(ELP_E_ARG, "elp_load_csc: more than 2^31-1 nonzeros");
    for (int64_t j = 0; j < n; ++j) {
        if (colptr[j + 1] < colptr[j]) return fail(ELP_E_ARG, "elp_load_csc: colptr must be nondecreasing");
        for (int64_t t = colptr[j]; t < colptr[j + 1]; ++t) {
            if (rowind[t] < 0 || rowind[t] >= m) return fail(ELP_E_ARG, "elp_load_csc: row index out of range");
            if (t > colptr[j] && rowind[t] <= rowind[t - 1])
                return fail(ELP_E_ARG, "elp_load_csc: row indices must be strictly increasing within a column");
            if (!std::isfinite(val[t])) return fail(ELP_E_ARG, "elp_load_csc: non-finite coefficient");
        }
    }
    int rc = prep_load(h, true);
    if (rc) return rc;
    std::vector<double> sval(val, val + nnz);  // scaled in place (scaling on)
    scale_csc(h, colptr, rowind, sval.data());
    val = sval.data();
    // CSR copy: a counting sort by row keeps the columns ascending within a row
    std::vector<int64_t> rp((size_t)m + 1, 0);
    for (int64_t t = 0; t < nnz; ++t) rp[(size_t)rowind[t] + 1]++;
    for (int64_t i = 0; i < m; ++i) rp[(size_t)i + 1] += rp[(size_t)i];
    std::vector<int32_t> ci((size_t)nnz);
    std::vector<double> rv((size_t)nnz);
    {
        std::vector<int64_t> next(rp.begin(), rp.end() - 1);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t t = colptr[j]; t < colptr[j + 1]; ++t) {
                const int64_t at = next[(size_t)rowind[t]]++;
                ci[(size_t)at] = (int32_t)j;
                rv[(size_t)at] = val[t];
            }
    }
    Dev& d = h->d;
    d.nnz = nnz;
    int64_t *dcp = nullptr, *drp = nullptr;
    int32_t *dri = nullptr, *dci = nullptr;
    double *dcv = nullptr, *drv = nullptr;
    HIPCHK(dalloc(&dcp, (size_t)n + 1));
    HIPCHK(dalloc(&dri, (size_t)nnz));
    HIPCHK(dalloc(&dcv, (size_t)nnz));
    HIPCHK(dalloc(&drp, (size_t)m + 1));
    HIPCHK(dalloc(&dci, (size_t)nnz));
    HIPCHK(dalloc(&drv, (size_t)nnz));
    d.cptr = dcp;
    d.rind = dri;
    d.cval = dcv;
    d.rptr = drp;
    d.cind = dci;
    d.rval = drv;
    HIPCHK(hipMemcpyAsync(dcp, colptr, ((size_t)n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, h->st));
    HIPCHK(hipMemcpyAsync(drp, rp.data(), ((size_t)m + 1) * sizeof(int64_t), hipMemcpyHostToDevice, h->st));
    if (nnz) {
        HIPCHK(hipMemcpyAsync(dri, rowind, (size_t)nnz * sizeof(int32_t), hipMemcpyHostToDevice, h->st));
        HIPCHK(hipMemcpyAsync(dcv, val, (size_t)nnz * sizeof(double), hipMemcpyHostToDevice, h->st));
        HIPCHK(hipMemcpyAsync(dci, ci.data(), (size_t)nnz * sizeof(int32_t), hipMemcpyHostToDevice, h->st));
        HIPCHK(hipMemcpyAsync(drv, rv.data(), (size_t)nnz * sizeof(double), hipMemcpyHostToDevice, h->st));
    }
    d.A = nullptr;
    rc = load_common(h, dir, rhs, obj, lo, up, maximize);
    HIPCHK(hipStreamSynchronize(h->st));  // the host CSR staging goes out of scope
    h->stats.seconds_load = now_s() - t0;
    return rc;
}

extern "C" int elp_load_generated(elp_handle* h, uint64_t seed) {
    if (is_group(h)) return fan_out(h, [&](elp_handle* r, int) { return elp_load_generated(r, seed); });
    const double t0 = now_s();
    int rc = prep_load(h);
    if (rc) return rc;
    const int64_t m = h->m, n = h->n;
    const int64_t c0 = h->replicated ? 0 : h->col0, nc = h->replicated ? n : h->nloc;
    HIPCHK(take_or_alloc(&h->A_owned, (size_t)m * (size_t)nc * sizeof(double), &h->keep_A, &h->keep_A_bytes));
    h->A_owned_bytes = (size_t)m * (size_t)nc * sizeof(double);
    double *db = nullptr, *dc = nullptr;
    HIPCHK(dalloc(&db, m));
    HIPCHK(dalloc(&dc, n));
    // generate this rank's shard of A (all of it when replicated) plus the full
    // b and c (c globally, for the objective)
    {
        Dev g = h->d;
        g.n = (int32_t)nc;
        HIPCHK(launch_generate(g, seed, c0, n, h->A_owned, db, nullptr, h->st));
        g.n = (int32_t)n;
        HIPCHK(launch_generate(g, seed, 0, n, nullptr, db, dc, h->st));
    }
    std::vector<double> b(m), c(n), lo(n, 0.0), up(n, HUGE_VAL);
    std::vector<int32_t> dir(m, ELP_LE);
    if (m) HIPCHK(hipMemcpyAsync(b.data(), db, m * sizeof(double), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipMemcpyAsync(c.data(), dc, n * sizeof(double), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    (void)hipFree(db);
    (void)hipFree(dc);
    rc = scale_dense(h, h->A_owned, c0, nc);
    if (rc) return rc;
    h->d.A = h->A_owned + (size_t)(h->col0 - c0) * (size_t)m;
    h->d.Afull = h->replicated ? h->A_owned : nullptr;
    rc = load_common(h, dir.data(), b.data(), c.data(), lo.data(), up.data(), 1);
    h->stats.seconds_load = now_s() - t0;
    return rc;
}

extern "C" int elp_generate_dense(int32_t device, uint64_t seed, int64_t m, int64_t n, double* dA,
                                  double* b, double* c) {
    if (m < 0 || n < 1 || m > 0x3fffffff || n > 0x3fffffff) return fail(ELP_E_ARG, "elp_generate_dense: bad size");
    if (m > 0 && !dA) return fail(ELP_E_ARG, "elp_generate_dense: dA is NULL");
    HIPCHK(hipSetDevice(device));
    hipStream_t st = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    double *db = nullptr, *dc = nullptr;
    hipError_t e = dalloc(&db, (size_t)(m > 0 ? m : 1));
    if (e == hipSuccess) e = dalloc(&dc, (size_t)n);
    Dev g{};
    g.m = (int32_t)m;
    g.n = (int32_t)n;
    if (e == hipSuccess) e = launch_generate(g, seed, 0, n, m > 0 ? dA : nullptr, db, dc, st);
    if (e == hipSuccess && b && m) e = hipMemcpyAsync(b, db, (size_t)m * sizeof(double), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess && c) e = hipMemcpyAsync(c, dc, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (db) (void)hipFree(db);
    if (dc) (void)hipFree(dc);
    (void)hipStreamDestroy(st);
    if (e != hipSuccess) return fail(ELP_E_HIP, std::string("elp_generate_dense: ") + hipGetErrorString(e));
    return 0;
}

static int push_ctl_fields(elp_handle* h) {
    // host-owned fields are written as one block (the device is idle at a poll)
    HIPCHK(hipMemcpyAsync(h->d.ctl, h->hctl, sizeof(DevCtl), hipMemcpyHostToDevice, h->st));
    return 0;
}

// Refactor at a poll: one Newton-Schulz correction of Minv when the residual
// of the maintained inverse is small, else a Gauss-Jordan rebuild; then the
// primal values from b (oracle/elp_oracle.c refactor()).
static int do_refactor(elp_handle* h, int k) {
    if (k > 0) {
        int rc = ensure_w(h, k);
        if (rc) return rc;
        // E = I - M Minv (its max |e| back to the host)
        auto resid = [&](double* emax) -> int {
            HIPCHK(hipMemsetAsync(&h->d.ctl->ns_emax_bits, 0, sizeof(unsigned long long), h->st));
            HIPCHK(launch_refactor_ns_resid(h->d, k, h->st));
            HIPCHK(hipMemcpyAsync(&h->hctl->ns_emax_bits, &h->d.ctl->ns_emax_bits, sizeof(unsigned long long),
                                  hipMemcpyDeviceToHost, h->st));
            HIPCHK(hipStreamSynchronize(h->st));
            const unsigned long long bits = h->hctl->ns_emax_bits;
            std::memcpy(emax, &bits, sizeof(*emax));
            if (h->ctl.refactor_mode == 0 && *emax > h->stats.max_inv_resid) h->stats.max_inv_resid = *emax;
            static const bool dbg = std::getenv("ELP_DEBUG_REFACTOR") != nullptr;
            if (dbg) std::fprintf(stderr, "elp refactor: k %d max|I - M Minv| %.3e\n", k, *emax);
            return 0;
        };
        double emax = 0.0;
        if (const int rc = resid(&emax)) return rc;
        bool ok = false;
        if (h->ctl.refactor_mode == 0 && emax <= NS_TOL) {
            HIPCHK(launch_refactor_ns_update(h->d, k, h->st));
            ok = true;
        } else if (h->ctl.refactor_mode == 0 && emax <= NS_TOL2) {  // (oracle refactor(): two corrections)
            HIPCHK(launch_refactor_ns_update(h->d, k, h->st));
            double e2 = 0.0;
            if (const int rc = resid(&e2)) return rc;
            if (e2 <= NS_TOL) {
                HIPCHK(launch_refactor_ns_update(h->d, k, h->st));
                ok = true;
            }
        }
        if (!ok) {
            HIPCHK(launch_refactor_gj(h->d, k, h->st));
            h->stats.gj_refactors++;
        }
    }
    HIPCHK(launch_nzlist(h->d, h->st));
    {
        const int rc = row_chain(h);
        if (rc) return rc;
    }
    HIPCHK(launch_refactor_primal(h->d, k, h->st));
    if (h->phase >= 2) HIPCHK(launch_btran_exact(h->d, k, h->st));  // exact duals again (phase 3: the dual's costs)
    h->stats.refactors++;
    return 0;
}

#ifdef ELP_PDBG
// diagnostic: the stamps of the last pricing launch of a chunk, appended to
// $ELP_PDBG_FILE at the first poll at or past each multiple of $ELP_PDBG_ITER
static void pdbg_dump(elp_handle* h, const DevCtl* c) {
    const char* fe = getenv("ELP_PDBG_FILE");
    const char* ie = getenv("ELP_PDBG_ITER");
    if (!fe || !ie || !h->d.ptimer || h->phase != 2 || c->status != ST_RUN) return;
    const int64_t every = atoll(ie);
    static int64_t next = 0;
    if (c->iter < next || every <= 0) return;
    next = (c->iter / every + 1) * every;
    const int grid = c->price_grid;
    std::vector<unsigned long long> v((size_t)6 * grid);
    if (hipMemcpy(v.data(), h->d.pstamp, v.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    unsigned long long t0 = ~0ull;
    for (int b = 0; b < grid; ++b) t0 = std::min(t0, v[6 * b]);
    FILE* f = fopen(fe, "a");
    if (!f) return;
    fprintf(f, "# iter %lld ny %d k %d grid %d ntiles %lld\n", (long long)c->iter, c->ny, c->k, grid,
            (long long)((h->n + TILE_COLS - 1) / TILE_COLS));
    for (int b = 0; b < grid; ++b) {
        const unsigned long long* r = &v[6 * b];
        const bool tile = r[1] > 16;
        auto rel = [&](int s) { return tile ? 10 * (long long)(r[s] - t0) : -1ll; };
        fprintf(f, "%d %s %lld %lld %lld %lld %lld %lld\n", b, tile ? "tile" : r[1] == 1 ? "apply" : "slack",
                10 * (long long)(r[0] - t0), rel(1), rel(2), rel(3), rel(4), 10 * (long long)(r[5] - t0));
    }
    fclose(f);
}
#endif

// The resident small-LP solver (elp_resident.hip): one GPU, no
// column shards, and the LP's whole state within the LDS one workgroup may
// allocate.  Returns the dynamic LDS bytes, 0 when not eligible.
static size_t resident_fit(elp_handle* h) {
    static const int env = [] {
        const char* e = std::getenv("ELP_RESIDENT");  // test hook: 0 never, 1 when it fits
        return e ? std::atoi(e) : -1;
    }();
    const int mode = env >= 0 ? (env == 0 ? 2 : 1) : h->ctl.resident;
    if (mode == 2 || h->comm.kind != 0 || h->d.sharded || h->m < 1 || h->nloc < 1 || h->nloc != h->n) return 0;
    if (h->res_lds_max == 0) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeSharedMemPerBlockOptin, h->dev) != hipSuccess || v <= 0) {
            (void)hipGetLastError();
            v = 65536;
        }
        h->res_lds_max = std::min<size_t>((size_t)v, (size_t)160 * 1024);
    }
    const size_t b = resident_lds_bytes((int)h->m, (int)h->n);
    return b <= h->res_lds_max ? b : 0;
}

// the pinned block's parts (elp_handle::res_pin), allocated at the first use
static constexpr size_t RES_PIN_X = (sizeof(ResOut) + 63) & ~(size_t)63;
static int ensure_res_pin(elp_handle* h) {
    if (!h->res_pin) HIPCHK(hipHostMalloc((void**)&h->res_pin, RES_PIN_X + 3 * (size_t)std::max<int64_t>(h->n, 1) * sizeof(double)));
    return 0;
}
static double* res_pin_x(elp_handle* h) { return reinterpret_cast<double*>(h->res_pin + RES_PIN_X); }

// One launch runs the loop to its end: optimal, infeasible, unbounded, a
// limit, or the elp_iterate budget (phase changes and refactors inside).
// Returns 1 when the pipeline must run instead (a plan still pending).
static int run_resident(elp_handle* h, size_t lds, int32_t* lp_status, double t_loop0) {
    DevCtl* c = h->hctl;
    if (c->plan_seq != c->applied_seq || c->copy_seq != c->plan_seq) return 1;
    int rc = ensure_ar(h, h->m);
    if (rc) return rc;
    rc = ensure_k(h, std::min(h->m, h->n));
    if (rc) return rc;
    if (!h->d_resout) HIPCHK(hipMalloc((void**)&h->d_resout, RES_PIN_X + (size_t)h->n * sizeof(double)));
    h->d_resx = reinterpret_cast<double*>(reinterpret_cast<char*>(h->d_resout) + RES_PIN_X);
    if (const int rp = ensure_res_pin(h)) return rp;
    ResArgs a{};
    a.phase = h->phase;
    a.price_rule = h->ctl.pricing;
    a.refactor_mode = h->ctl.refactor_mode;
    a.warm = h->res_warm;
    a.xout = h->d_resx;
    a.tick_budget = 0;
    if (h->ctl.time_limit > 0) {
        const double left = h->ctl.time_limit - (now_s() - h->t_solve_start);
        a.tick_budget = std::max<int64_t>(1, (int64_t)(left * 1e8));
    }
    a.out = h->d_resout;
    HIPCHK(launch_resident(h->d, a, lds, h->st));
    ResOut o{};
    HIPCHK(hipMemcpyAsync(c, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipMemcpyAsync(h->res_pin, h->d_resout, RES_PIN_X + (size_t)h->n * sizeof(double), hipMemcpyDeviceToHost,
                          h->st));  // (the record and x together: the pinned block's layout)
    HIPCHK(hipStreamSynchronize(h->st));
    std::memcpy(&o, h->res_pin, sizeof(ResOut));
    h->res_x.assign(res_pin_x(h), res_pin_x(h) + h->n);
    h->res_fresh = true;
    h->stats.host_polls++;
    // (a warm start's refactor is not counted: reload_bounds_warm resets the count after it)
    h->stats.refactors += std::max<int64_t>(0, o.refactors - (a.warm ? 1 : 0));
    h->res_warm = 0;
    h->stats.gj_refactors += o.gj_refactors;
    if (h->ctl.refactor_mode == 0 && o.emax_max > h->stats.max_inv_resid) h->stats.max_inv_resid = o.emax_max;
    h->stats.resident = 1;
    h->stats.resident_launches++;
    h->stats.resident_ticks += o.ticks;
    if (o.stage[1] && std::getenv("ELP_DEBUG_RESIDENT"))  // (a -DELP_RES_PROF=1 build)
        std::fprintf(stderr, "elp resident: %lld iterations, shader cycles top+btran %lld select %lld ftran %lld "
                     "finish %lld basis %lld refactor %lld loop %lld; kernel %.1f us\n", (long long)c->iter,
                     (long long)o.stage[0], (long long)o.stage[1], (long long)o.stage[2], (long long)o.stage[3],
                     (long long)o.stage[4], (long long)o.stage[5], (long long)o.stage[7], o.ticks / 100.0);
    if (o.stage[1] && std::getenv("ELP_DEBUG_RESIDENT"))
        std::fprintf(stderr, "elp resident inner: ftran colA+shf %lld wdot %lld zchunk %lld; price loop %lld argbest %lld; "
                     "ratio pass1 %lld pass2 %lld\n", (long long)o.stage2[0], (long long)o.stage2[1], (long long)o.stage2[2],
                     (long long)o.stage2[3], (long long)o.stage2[4], (long long)o.stage2[5], (long long)o.stage2[6]);
    if (o.stage[1] && std::getenv("ELP_DEBUG_RESIDENT"))
        std::fprintf(stderr, "elp resident dual select: chuzr %lld rho %lld sweep %lld compaction %lld bfrt %lld flips %lld\n",
                     (long long)o.stage3[0], (long long)o.stage3[1], (long long)o.stage3[2], (long long)o.stage3[3],
                     (long long)o.stage3[4], (long long)o.stage3[5]);
    h->phase = o.phase;
    const int32_t s = c->status;
    h->stats.seconds_loop += now_s() - t_loop0;
    if (s == ST_STOP) {
        c->status = ST_RUN;
        *lp_status = ELP_SUBOPTIMAL;
        return push_ctl_fields(h);
    }
    h->done = true;
    if (s == ST_PHASE_OPT) h->final_status = h->phase == 1 ? ELP_INFEASIBLE : ELP_OPTIMAL;
    else if (s == ST_UNBOUNDED) h->final_status = ELP_UNBOUNDED;
    else if (s == ST_DUALINF) h->final_status = ELP_INFEASIBLE;
    else if (s == ST_ITERCAP) h->final_status = ELP_SUBOPTIMAL;
    else if (s == ST_TIMEOUT) h->final_status = ELP_TIMEOUT;
    else h->final_status = ELP_NUMFAILURE;
    *lp_status = h->final_status;
    return 0;
}

// the polling loop; budget = iterations allowed in this call
static int run_loop(elp_handle* h, int64_t budget, int32_t* lp_status) {
    if (h->done) {
        *lp_status = h->final_status;
        return 0;
    }
    const double t_loop0 = now_s();
    if (!h->timing_started) {
        h->t_solve_start = t_loop0;
        h->timing_started = true;
    }
    DevCtl* c = h->hctl;
    // resume: refresh the mirror (unless it is the device's already), set the stop budget
    if (!h->res_fresh && !h->ctl_fresh) {
        HIPCHK(hipMemcpyAsync(c, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
        HIPCHK(hipStreamSynchronize(h->st));
    }
    h->res_fresh = false;
    h->ctl_fresh = false;
    c->iter_stop = budget >= INT64_MAX - c->iter ? INT64_MAX : c->iter + budget;
    if (c->status == ST_STOP) c->status = ST_RUN;
    c->phase = h->phase;
    int rc = push_ctl_fields(h);
    if (rc) return rc;
    if (const size_t lds = resident_fit(h)) {
        rc = run_resident(h, lds, lp_status, t_loop0);
        if (rc != 1) return rc;
    }
    if (h->res_warm)  // (reload_bounds_warm took the resident path: its device part is the kernel's)
        return fail(ELP_E_STATE, "internal: a resident warm start fell back to the pipeline");
    h->stats.resident = 0;
    const int period = h->ctl.refactor_period;
    // ELP_PROFILE_EVENTS: events on the pricing dispatches of every chunk;
    // ELP_PROFILE_SAMPLE: of every 8th chunk only (a uniform sample of the solve
    // that leaves the other chunks' dispatches untouched)
    const bool prof_all = (h->ctl.verbose & ELP_PROFILE_EVENTS) != 0;
    const bool prof = prof_all || (h->ctl.verbose & ELP_PROFILE_SAMPLE) != 0;
    if (prof && (int)h->ev.size() < 2 * h->ctl.sync_every) {
        for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
        h->ev.assign(2 * h->ctl.sync_every, nullptr);
        for (auto& e : h->ev) HIPCHK(hipEventCreate(&e));
    }
    for (;;) {
        // host-side loop-top work at a poll (no launch is wasted on it):
        // budget exhausted -> return; refactor due (phase 2) -> do it now.
        if (c->status == ST_RUN && c->iter >= c->iter_stop && c->iter < c->iter_limit) {
            *lp_status = ELP_SUBOPTIMAL;
            h->stats.seconds_loop += now_s() - t_loop0;
            return 0;
        }
        if (c->status == ST_RUN && h->phase >= 2 && c->iter >= c->iter_limit) {
            // the phase-2 loop top (oracle run_phase) before any k_ratio has
            // checked the cap: a budget spent in phase 1 or a branch-and-bound
            // budget of 0
            h->done = true;
            h->final_status = ELP_SUBOPTIMAL;
            break;
        }
        if (c->status == ST_RUN && h->phase >= 2 && c->since_refactor >= period &&
            c->iter < c->iter_limit) {
            rc = do_refactor(h, c->k);
            if (rc) return rc;
            HIPCHK(hipMemcpyAsync(c, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
            HIPCHK(hipStreamSynchronize(h->st));
            if (c->status == ST_NUMFAIL) {
                h->done = true;
                h->final_status = ELP_NUMFAILURE;
                break;
            }
            c->since_refactor = 0;
            rc = push_ctl_fields(h);
            if (rc) return rc;
        }
        const int k0 = c->k, ny0 = c->ny;
        int chunk = h->ctl.sync_every;
        rc = ensure_ar(h, (int64_t)ny0 + chunk + 1);  // |Y| grows by <= 1 per iteration
        if (rc) return rc;
        rc = ensure_k(h, (int64_t)k0 + chunk + 2);  // so does k
        if (rc) return rc;
        const int to_refactor = period - c->since_refactor;
        if (to_refactor > 0 && to_refactor < chunk) chunk = to_refactor;
        const int64_t left = c->iter_stop - c->iter;
        if (left > 0 && left < chunk) chunk = (int)left;
        if (chunk < 1) chunk = 1;
        const double bytes0 = c->price_bytes;
        if (h->d.dstamp) {  // debug: min-start slot at +inf, maxima at 0
            std::vector<unsigned long long> init(DSTAMP_STRIDE * 64, 0ull);
            for (int t = 0; t < 64; ++t) init[t * DSTAMP_STRIDE + 11] = ~0ull;
            HIPCHK(hipMemcpyAsync(h->d.dstamp, init.data(), init.size() * 8, hipMemcpyHostToDevice, h->st));
            HIPCHK(hipStreamSynchronize(h->st));
        }
        const double t_enq0 = now_s();
        const bool prof_chunk = prof && (prof_all || h->prof_chunks++ % 8 == 0);
        // (the device-clock timer of the same launches: ticks before the chunk)
        const unsigned long long ticks0 = c->price_ticks;
        const int64_t timed0 = c->price_timed;
        for (int t = 0; t < chunk; ++t) {
            const int kub = (int)std::min<int64_t>(h->m, (int64_t)k0 + t);
            const int nyub = (int)std::min<int64_t>(h->m, (int64_t)ny0 + t);
            hipEvent_t e0 = prof_chunk ? h->ev[2 * t] : nullptr, e1 = prof_chunk ? h->ev[2 * t + 1] : nullptr;
            h->stats.price_launches++;
            if (h->phase == 3 && h->comm.kind == 0) {  // the dual simplex phase 1 (one GPU)
                HIPCHK(launch_dual_iteration(h->d, kub, nyub, h->st, t));
            } else if (h->phase == 3) {
                // column-sharded: each rank prices its shard (the last rank also the
                // slacks) and packs its ratio-test candidates; the all-gather hands
                // every rank all of them in rank order, and every rank runs the same
                // bound-flipping ratio test and update
                HIPCHK(launch_dual_iteration_head(h->d, kub, nyub, h->st));
                rc = h->comm.allgather(h->d.dsend, h->d.drecv, ((size_t)h->d.dcap + 1) * sizeof(DualCand), h->st);
                if (rc) return fail(rc, "dual ratio-test candidate all-gather failed");
                if (h->replicated) {
                    HIPCHK(launch_dual_iteration_tail(h->d, kub, h->st));
                } else {
                    // column-only shards: the entering column travels (all-reduce of
                    // the owner's copy), and a_F = sum of the flipped columns is one
                    // per-row chain continued shard after shard (a broadcast each)
                    HIPCHK(launch_dual_ratio_shards(h->d, h->st));
                    rc = h->comm.allreduce_sum_f64(h->d.pkt, (size_t)h->m, h->st);
                    if (rc) return fail(rc, "entering-column all-reduce failed");
                    for (int r = 0; r < h->comm.world; ++r) {
                        if (r == h->comm.rank) HIPCHK(launch_dual_flip_part(h->d, h->st));
                        rc = h->comm.bcast_f64(h->d.aF, (size_t)h->m, r, h->st);
                        if (rc) return fail(rc, "bound-flip column broadcast failed");
                    }
                    HIPCHK(launch_dual_iteration_finish(h->d, kub, h->st));
                }
            } else if (h->comm.kind == 0 || h->d.p2p) {  // (p2p: min-loc inside the select kernel)
                HIPCHK(launch_iteration(h->d, kub, nyub, h->phase, h->st, e0, e1, t, prof_chunk ? t : -1));
            } else {
                // sharded: local min-loc -> all-gather -> global min-loc.  Replicated
                // A: a_R + bump FTRAN straight from the local copy -> tail.  Else the
                // owner packs its column, all-reduce (non-owners contribute zeros).
                HIPCHK(launch_iteration_head(h->d, kub, nyub, h->phase, h->comm.rank, h->st, e0, e1,
                                             prof_chunk ? t : -1));
                rc = h->comm.allgather(h->d.cand_xchg + h->comm.rank, h->d.cand_xchg, sizeof(CandX), h->st);
                if (rc) return fail(rc, "candidate all-gather failed");
                if (h->replicated) {
                    hipError_t le = hipSuccess;
                    if (launch_select_xftran(h->d, kub, h->st, &le)) {
                        HIPCHK(le);
                        HIPCHK(launch_iteration_tail(h->d, kub, h->phase, h->st, false));
                        continue;
                    }
                    HIPCHK(launch_select_global(h->d, h->st));
                    HIPCHK(launch_select_finish(h->d, h->st));
                    HIPCHK(launch_iteration_tail(h->d, kub, h->phase, h->st));
                    continue;
                }
                HIPCHK(launch_select_global(h->d, h->st));
                rc = h->comm.allreduce_sum_f64(h->d.pkt, (size_t)h->m + 4, h->st);
                if (rc) return fail(rc, "entering-column all-reduce failed");
                HIPCHK(launch_select_finish(h->d, h->st));
                HIPCHK(launch_iteration_tail(h->d, kub, h->phase, h->st));
            }
        }
        const double t_enq1 = now_s();
        if (prof_chunk && h->phase == 2) HIPCHK(launch_ptimer_reduce(h->d, std::min(chunk, h->d.ptslots), h->st));
        HIPCHK(hipMemcpyAsync(c, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
        HIPCHK(hipStreamSynchronize(h->st));
        // a poll that just queues the next chunk (phase 2 running, no budget, cap,
        // refactor or time-limit stop due) leaves the last plan to the next chunk's
        // first pricing launch, as inside a chunk; any other poll may read the basis
        const bool ddefer = h->phase == 3 && h->comm.kind == 0 && h->d.dual_defer;
        const bool plain_next = c->status == ST_RUN && (h->phase == 2 || ddefer) && c->iter < c->iter_stop &&
                                c->iter < c->iter_limit && c->since_refactor < period && !(h->ctl.time_limit > 0);
        if ((c->plan_seq != c->applied_seq || (ddefer && c->plan_seq != c->copy_seq)) && !plain_next) {
            // phase 2 defers each iteration's update into the next pricing launch,
            // the one-GPU dual phase into the next iteration's launches: apply the
            // last one now (phase 1 and sharded dual ranks applied theirs in place)
            if (h->phase == 2) HIPCHK(launch_apply_pending(h->d, std::max(k0, c->k), h->st));
            if (ddefer) HIPCHK(launch_apply_pending(h->d, std::max(k0, c->k) + 1, h->st, true));
            c->applied_seq = c->copy_seq = c->plan_seq;
            rc = push_ctl_fields(h);
            if (rc) return rc;
        }
        h->dbg_enqueue += t_enq1 - t_enq0;
        if (h->d.dstamp && c->status == ST_RUN && (h->phase == 2 || h->phase == 3)) {
            std::vector<unsigned long long> v(DSTAMP_STRIDE * 64);
            HIPCHK(hipMemcpy(v.data(), h->d.dstamp, v.size() * 8, hipMemcpyDeviceToHost));
            if (h->stamp_sum.empty()) h->stamp_sum.assign(DSTAMP_STRIDE + 24, 0.0);
            for (int t = 0; t < chunk; ++t) {
                const unsigned long long* r = &v[(size_t)t * DSTAMP_STRIDE];
                // time base: the first workgroup's start (ELP_STAMPS=2), else workgroup 0's
                const unsigned long long base = r[11] != ~0ull ? r[11] : r[0];
                for (int i = 0; i < 11; ++i)
                    if (r[i]) h->stamp_sum[i] += 10.0 * (double)(long long)(r[i] - base);  // ns (100 MHz)
                for (int i = 13; i < 16; ++i)  // select kernel, relative to its workgroup 0's start
                    if (r[i] && r[12]) h->stamp_sum[i] += 10.0 * (double)(long long)(r[i] - r[12]);
                for (int i = 17; i < 20; ++i)  // FTRAN-z, relative to its workgroup 0's start
                    if (r[i] && r[16]) h->stamp_sum[i] += 10.0 * (double)(long long)(r[i] - r[16]);
                for (int i = 21; i < 24; ++i)  // the dual BFRT, relative to its start
                    if (r[i] && r[20]) h->stamp_sum[i] += 10.0 * (double)(long long)(r[i] - r[20]);
                for (int i : {27, 29, 30, 31, 32, 33})  // (conditional: counted where present, in stamp_sum[34 + ...])
                    if (r[i] && r[20] && r[i] >= r[20] && r[i] - r[20] < 100000ull) {
                        h->stamp_sum[i] += 10.0 * (double)(long long)(r[i] - r[20]);
                        h->stamp_sum[i == 27 ? 34 : i == 29 ? 35 : 36] += i < 30 || i == 30 ? 1.0 : 0.0;
                    }
                for (int i : {24, 25, 26, 28}) h->stamp_sum[i] += (double)r[i];  // (counts)
                if (r[30] && r[20] && r[29] >= r[20] && r[23] >= r[20] && r[30] - r[20] < 100000ull) {
                    // the launches whose fast tail ran (flips): every phase over the same launches
                    int s = 40;
                    for (int i : {21, 27, 29, 22, 30, 23}) h->stamp_sum[s++] += 10.0 * (double)(long long)(r[i] - r[20]);
                    h->stamp_sum[46] += (double)r[24];
                    h->stamp_sum[47] += (double)r[28];
                    h->stamp_sum[48] += 1.0;
                }
                if (r[36] >= 1 && r[36] <= 3 && r[23] >= r[20] && r[23] - r[20] < 100000ull) {
                    // per a_F path (1 one wave, 2 LDS block, 3 column walk): launches, end, entries
                    const int b = 49 + 3 * (int)(r[36] - 1);
                    h->stamp_sum[b] += 1.0;
                    h->stamp_sum[b + 1] += 10.0 * (double)(r[23] - r[20]);
                    h->stamp_sum[b + 2] += (double)(long long)r[35];
                }
                if (r[34] && r[23] > r[20]) {  // the BFRT launch's shader clock: s_memtime ticks per 10 ns
                    h->stamp_sum[37] += (double)r[34];
                    h->stamp_sum[38] += 10.0 * (double)(r[23] - r[20]);
                }
                h->stamp_n++;
            }
        }
        h->dbg_wait += now_s() - t_enq1;
        h->stats.host_polls++;
#ifdef ELP_PDBG
        pdbg_dump(h, c);
#endif
        const int32_t s = c->status;
        if (s == ST_COMMFAIL)
            return fail(ELP_E_COMM, "xGMI mailbox: a peer's record did not arrive within elp_control.mailbox_timeout");
        if (prof_chunk && s == ST_RUN) {  // every launch of the chunk did work
            for (int t = 0; t < chunk; ++t) {
                float ms = 0.f;
                HIPCHK(hipEventElapsedTime(&ms, h->ev[2 * t], h->ev[2 * t + 1]));
                h->stats.price_seconds += 1e-3 * ms;
            }
            h->stats.price_timed_launches += chunk;
            h->stats.price_timed_bytes += c->price_bytes - bytes0;
            h->stats.price_seconds_stamps += 1e-8 * (double)(c->price_ticks - ticks0);  // (100 MHz clock)
            h->stats.price_stamped_launches += c->price_timed - timed0;
        }
        if (s == ST_RUN) {
            if (h->ctl.time_limit > 0) {
                int over = 0;
                rc = any_rank(h, now_s() - h->t_solve_start > h->ctl.time_limit, &over);
                if (rc) return rc;
                if (over) {
                    h->done = true;
                    h->final_status = ELP_TIMEOUT;
                    break;
                }
            }
            continue;
        }
        if (s == ST_REFACTOR) {
            rc = do_refactor(h, c->k);
            if (rc) return rc;
            HIPCHK(hipMemcpyAsync(c, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
            HIPCHK(hipStreamSynchronize(h->st));
            if (c->status == ST_NUMFAIL) {
                h->done = true;
                h->final_status = ELP_NUMFAILURE;
                break;
            }
            c->since_refactor = 0;
            c->status = ST_RUN;
            rc = push_ctl_fields(h);
            if (rc) return rc;
            continue;
        }
        if (s == ST_STOP) {
            *lp_status = ELP_SUBOPTIMAL;
            h->stats.seconds_loop += now_s() - t_loop0;
            return 0;
        }
        if (s == ST_DUALINF && h->phase == 3) {  // the dual ray: no nonbasic can repair the leaving row
            h->done = true;
            h->final_status = ELP_INFEASIBLE;
            break;
        }
        if (s == ST_PHASE_OPT && h->phase == 3) {
            // primal feasible: confirm on a fresh x_B after updates (oracle run_dual),
            // else the real costs and the primal phase 2 from this basis
            const bool recheck = c->since_refactor > 0;
            if (!recheck) {
                HIPCHK(launch_phase2(h->d, h->st));
                h->phase = 2;
            }
            rc = do_refactor(h, c->k);
            if (rc) return rc;
            HIPCHK(hipMemcpyAsync(c, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
            HIPCHK(hipStreamSynchronize(h->st));
            if (c->status == ST_NUMFAIL) {
                h->done = true;
                h->final_status = ELP_NUMFAILURE;
                break;
            }
            c->phase = 2;
            c->since_refactor = 0;
            if (!recheck) {
                c->ndegen = 0;
                c->bland = 0;
                c->devex = h->ctl.pricing == ELP_PRICE_DEVEX;
            }
            c->status = ST_RUN;
            rc = push_ctl_fields(h);
            if (rc) return rc;
            continue;
        }
        if ((s == ST_PHASE_OPT || s == ST_P1DONE) && h->phase == 1) {
            if (s == ST_PHASE_OPT && c->art_sum > c->tol_inf) {
                h->done = true;
                h->final_status = ELP_INFEASIBLE;
                break;
            }
            HIPCHK(launch_phase2(h->d, h->st));
            h->phase = 2;
            rc = do_refactor(h, c->k);
            if (rc) return rc;
            HIPCHK(hipMemcpyAsync(c, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
            HIPCHK(hipStreamSynchronize(h->st));
            if (c->status == ST_NUMFAIL) {
                h->done = true;
                h->final_status = ELP_NUMFAILURE;
                break;
            }
            c->phase = 2;
            c->since_refactor = 0;
            c->ndegen = 0;
            c->bland = 0;
            c->status = ST_RUN;
            rc = push_ctl_fields(h);
            if (rc) return rc;
            continue;
        }
        if (s == ST_PHASE_OPT && h->phase == 2 && c->since_refactor > 0) {
            // optimal under updated duals: refactor (exact y) and price again
            rc = do_refactor(h, c->k);
            if (rc) return rc;
            HIPCHK(hipMemcpyAsync(c, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
            HIPCHK(hipStreamSynchronize(h->st));
            if (c->status == ST_NUMFAIL) {
                h->done = true;
                h->final_status = ELP_NUMFAILURE;
                break;
            }
            c->since_refactor = 0;
            c->status = ST_RUN;
            rc = push_ctl_fields(h);
            if (rc) return rc;
            continue;
        }
        h->done = true;
        if (s == ST_PHASE_OPT) h->final_status = ELP_OPTIMAL;
        else if (s == ST_UNBOUNDED) h->final_status = ELP_UNBOUNDED;
        else if (s == ST_ITERCAP) h->final_status = ELP_SUBOPTIMAL;
        else h->final_status = ELP_NUMFAILURE;
        break;
    }
    h->stats.seconds_loop += now_s() - t_loop0;
    *lp_status = h->final_status;
    return 0;
}

extern "C" int elp_set_int(elp_handle* h, const int32_t* is_int) {
    if (is_group(h)) return fan_out(h, [&](elp_handle* r, int) { return elp_set_int(r, is_int); }, false);
    if (!h || !h->loaded) return fail(ELP_E_STATE, "elp_set_int: no problem loaded");
    h->is_int.clear();
    if (is_int) {
        bool any = false;
        for (int64_t j = 0; j < h->n; ++j) any |= is_int[j] != 0;
        if (any) h->is_int.assign(is_int, is_int + h->n);
    }
    return 0;
}

// reload the LP with column bounds lo / up (a branch-and-bound node): A, rows
// and objective stay; the device state restarts from the slack basis
static int reload_bounds(elp_handle* h, const std::vector<double>& lo, const std::vector<double>& up) {
    const std::vector<int32_t> dir = h->dir_h;
    const std::vector<double> rhs = h->rhs_h, obj = h->obj_h;
    h->in_bnb = true;
    int rc = load_common(h, dir.data(), rhs.data(), obj.data(), lo.data(), up.data(), h->maximize);
    h->in_bnb = false;
    return rc;
}

// A branch-and-bound node warm-started from the basis the last node ended on
// (oracle warm_core; SIMPLEX_DUAL_PRIMAL on one GPU): the node's bounds, the
// real costs, every nonbasic column re-placed for them (launch_warm_start), a
// refactor (Minv correction, x_B from b), then the dual phase 1 from that
// basis -- its first CHUZR ends it at once when x_B is feasible -- and the
// primal phase 2.  Device memory, A, the rows and the lists all stay.
static int reload_bounds_warm(elp_handle* h, const std::vector<double>& lo, const std::vector<double>& up) {
    const int64_t n = h->n;
    Dev& d = h->d;
    const double BIG = h->ctl.infinity;
    auto fin = [&](double v) { return v <= -BIG ? -HUGE_VAL : v >= BIG ? HUGE_VAL : v; };
    std::vector<double> lo_s((size_t)n), up_s((size_t)n);
    for (int64_t j = 0; j < n; ++j) {
        lo_s[(size_t)j] = unscale_col(h, fin(lo[(size_t)j]), j, -1);
        up_s[(size_t)j] = unscale_col(h, fin(up[(size_t)j]), j, -1);
    }
    // the last node ran on the resident solver and nothing ran since: the
    // mirror is the device's control block, and the next resident launch does
    // the device part (launch_warm_start, do_refactor, the weights' reset)
    const bool res = h->res_fresh && resident_fit(h) != 0;
    h->res_fresh = false;
    double *dlo = d.lb, *dup = d.ub;  // (res: the structurals' bounds in place)
    const double *src_lo = lo_s.data(), *src_up = up_s.data();
    if (res) {  // (from the pinned block: an asynchronous copy)
        if (const int rp = ensure_res_pin(h)) return rp;
        double* pl = res_pin_x(h) + n;
        std::memcpy(pl, lo_s.data(), (size_t)n * sizeof(double));
        std::memcpy(pl + n, up_s.data(), (size_t)n * sizeof(double));
        src_lo = pl;
        src_up = pl + n;
    } else {
        if (!h->warm_lo) HIPCHK(hipMalloc((void**)&h->warm_lo, (size_t)std::max<int64_t>(n, 1) * sizeof(double)));
        if (!h->warm_up) HIPCHK(hipMalloc((void**)&h->warm_up, (size_t)std::max<int64_t>(n, 1) * sizeof(double)));
        dlo = h->warm_lo;
        dup = h->warm_up;
    }
    HIPCHK(hipMemcpyAsync(dlo, src_lo, (size_t)n * sizeof(double), hipMemcpyHostToDevice, h->st));
    HIPCHK(hipMemcpyAsync(dup, src_up, (size_t)n * sizeof(double), hipMemcpyHostToDevice, h->st));
    // the control block of a fresh solve, the basis kept
    if (!res) {
        HIPCHK(hipMemcpyAsync(h->hctl, d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
        HIPCHK(hipStreamSynchronize(h->st));
    }
    DevCtl& c = *h->hctl;
    const int k = c.k, ny = c.ny;
    c.status = ST_RUN;
    c.phase = 2;
    c.iter = 0;
    // a new mailbox epoch, as every load: the iteration count restarts at 0, and
    // the last node's final records (seq = epoch << 40 | iteration + 1) still sit
    // in the peers' slots -- under the old epoch a rank reaching the same
    // iteration number could take a stale record for its peer's
    c.mb_epoch = ++h->mb_epoch;
    c.iter_limit = h->ctl.max_iter > 0 ? std::max<int64_t>(h->bnb_iter_left, 0) : 100 * (h->m + n) + 10000;
    c.iter_stop = INT64_MAX;
    c.since_refactor = 0;
    c.ndegen = c.bland = 0;
    c.phase1_iters = c.flips = c.degenerate = 0;
    c.unb_var = -1;
    c.infeasible_bounds = 0;
    c.price_bytes = c.iter_bytes = 0.0;
    c.price_passes = 0;
    c.plan.action = ACT_NONE;
    c.plan_seq = c.applied_seq = c.copy_seq = 0;
    c.devex = 0;
    c.ddevex = h->ctl.pricing == ELP_PRICE_DEVEX;
    c.dv_valid = 0;
    c.dual_iters = c.dflat = 0;
    if (res) {
        bool bad = false;  // (k_warm_bounds' test, on the host's copy)
        for (int64_t j = 0; j < n; ++j) bad |= lo_s[(size_t)j] > up_s[(size_t)j];
        h->stats = elp_stats{};
        h->stats.world_size = h->comm.world;
        h->stats.ncols = h->nloc;
        h->stats.basis = ELP_BASIS_INVERSE;
        h->timing_started = false;
        h->done = false;
        h->dual_used = true;
        if (bad) {  // (the oracle's warm_core: nothing of the node runs)
            h->done = true;
            h->final_status = ELP_INFEASIBLE;
        } else {
            h->phase = 3;
            h->res_warm = 1;
        }
        const int rc = push_ctl_fields(h);
        if (rc) return rc;
        h->res_fresh = true;  // (the mirror was just written to the device)
        return 0;
    }
    HIPCHK(hipMemcpyAsync(d.ctl, h->hctl, sizeof(DevCtl), hipMemcpyHostToDevice, h->st));
    HIPCHK(launch_warm_start(d, dlo, dup, k, ny, h->st));
    HIPCHK(hipMemcpyAsync(h->hctl, d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    h->stats = elp_stats{};
    h->stats.world_size = h->comm.world;
    h->stats.ncols = h->nloc;
    h->stats.basis = ELP_BASIS_INVERSE;
    h->timing_started = false;
    h->done = false;
    h->dual_used = true;
    if (h->hctl->infeasible_bounds) {  // R/class.R:297-298 (as load_common)
        h->done = true;
        h->final_status = ELP_INFEASIBLE;
        return 0;
    }
    h->phase = 3;
    int rc = do_refactor(h, k);
    if (rc) return rc;
    HIPCHK(launch_devex_reset(d, h->st));  // (the dual phase's weights start at 1)
    HIPCHK(hipMemcpyAsync(h->hctl, d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    h->hctl->since_refactor = 0;
    h->hctl->dv_valid = 0;
    h->stats.refactors = 0;
    return push_ctl_fields(h);
}

// Depth-first branch and bound over LP relaxations; the rules are
// oracle/elp_oracle.c orc_solve_mip's, so both explore the same tree.
// max_iter (total LP iterations) and time_limit (seconds since the branch and
// bound started) bound the whole tree.  A node LP that stops on a limit ends
// the search; one that fails numerically is skipped but makes the result
// incomplete.  Status: unbounded relaxation -> 3; incumbent -> 0, or 1 when the
// tree was not fully explored (a limit, max_nodes, a failed node); no
// incumbent -> the failed node's status (1 iteration cap, 5, 7), 1 at the node
// limit, else 2 (lp_solve's SUBOPTIMAL / TIMEOUT / NUMFAILURE conventions).
static int run_bnb(elp_handle* h, int32_t* out_status) {
    const int64_t n = h->n;
    const double INF = HUGE_VAL, BIG = h->ctl.infinity;
    const double t_bnb = now_s();
    std::vector<double> l0 = h->lo_h, u0 = h->up_h;
    for (int64_t j = 0; j < n; ++j) {
        if (l0[j] <= -BIG) l0[j] = -INF;
        if (u0[j] >= BIG) u0[j] = INF;
        if (h->is_int[j]) {
            if (l0[j] > -INF) l0[j] = std::ceil(l0[j] - 1e-9);
            if (u0[j] < INF) u0[j] = std::floor(u0[j] + 1e-9);
        }
    }
    struct Node { std::vector<double> lo, up; };
    std::vector<Node> stack;
    stack.push_back({l0, u0});
    double best = INF;
    Node best_node;
    bool have = false, limit = false, unbounded = false;
    int32_t failed = -1;  // status of the first node LP that did not finish (incomplete tree)
    int64_t nodes = 0, iters = 0;
    std::vector<double> x((size_t)n), best_x;
    // SIMPLEX_DUAL_PRIMAL on one GPU: node LPs after the first continue from
    // the basis of the node solved last (reload_bounds_warm; oracle warm_core)
    const bool warm = dual_phase1(h) && h->m > 0;
    bool warm_ok = false;
    while (!stack.empty()) {
        Node nd = std::move(stack.back());
        stack.pop_back();
        if (h->ctl.max_nodes > 0 && nodes >= h->ctl.max_nodes) {
            limit = true;
            continue;
        }
        if (h->ctl.time_limit > 0) {
            // (a node LP checks the clock at its polls; small nodes finish
            // before their first poll, so the tree checks it between nodes too;
            // all ranks of a sharded solve take the same decision)
            int over = 0;
            const int rc = any_rank(h, now_s() - t_bnb > h->ctl.time_limit, &over);
            if (rc) return rc;
            if (over) {
                failed = failed < 0 ? ELP_TIMEOUT : failed;
                break;
            }
        }
        nodes++;
        h->bnb_iter_left = h->ctl.max_iter - iters;
        if (h->ctl.max_iter > 0 && h->bnb_iter_left <= 0) {  // budget spent: as the oracle
            failed = failed < 0 ? ELP_SUBOPTIMAL : failed;
            break;
        }
        int rc = 0;
        if (warm_ok && nodes > 1) rc = reload_bounds_warm(h, nd.lo, nd.up);
        else if (!(nodes == 1 && h->lo_h == nd.lo && h->up_h == nd.up)) rc = reload_bounds(h, nd.lo, nd.up);
        if (rc) return rc;
        h->t_solve_start = t_bnb;  // time_limit counts from the start of the tree
        h->timing_started = true;
        int32_t s = 0;
        rc = run_loop(h, INT64_MAX, &s);
        if (rc) return rc;
        {
            elp_stats st{};
            rc = elp_get_stats(h, &st);
            if (rc) return rc;
            iters += st.iterations;
        }
        if (s == ELP_UNBOUNDED) {
            unbounded = true;
            break;
        }
        // (the oracle: a node that failed leaves no basis to continue from -- the
        //  next one starts cold; so does a node the primal phase 1 solved)
        warm_ok = warm && (s == ELP_OPTIMAL || s == ELP_INFEASIBLE || s == ELP_UNBOUNDED);
        if (s != ELP_OPTIMAL && s != ELP_INFEASIBLE) {  // limit or numerical failure
            if (failed < 0) failed = s;
            if (s == ELP_SUBOPTIMAL || s == ELP_TIMEOUT) break;  // the tree's budget is spent
            continue;
        }
        if (s != ELP_OPTIMAL) continue;
        double z = 0.0;
        rc = elp_get_solution(h, &z, x.data(), nullptr, nullptr);
        if (rc) return rc;
        const double zmin = h->maximize ? -z : z;
        const double tol = std::fabs(best) < INF ? std::max(1e-11, 1e-9 * std::fabs(best)) : 0.0;
        if (std::fabs(best) < INF && zmin >= best - tol) continue;
        int64_t jb = -1;
        for (int64_t j = 0; j < n; ++j)
            if (h->is_int[j] && std::fabs(x[j] - std::nearbyint(x[j])) > 1e-7) {
                jb = j;
                break;
            }
        if (jb < 0) {
            best = zmin;
            best_node = nd;
            best_x = x;
            have = true;
            continue;
        }
        Node fl = nd;  // floor child pushed first: the ceiling child is explored first
        fl.up[jb] = std::floor(x[jb]);
        nd.lo[jb] = std::ceil(x[jb]);
        stack.push_back(std::move(fl));
        stack.push_back(std::move(nd));
    }
    int32_t status;
    if (unbounded) status = ELP_UNBOUNDED;
    else if (have) status = (limit || failed >= 0) ? ELP_SUBOPTIMAL : ELP_OPTIMAL;
    else if (failed >= 0) status = failed;
    else status = limit ? ELP_SUBOPTIMAL : ELP_INFEASIBLE;
    (void)best_node;
    // elp_get_solution reports the incumbent as the tree found it (the oracle's
    // xbest): no re-solve, whose warm start could end on another optimal vertex
    h->mip_x.clear();
    if (have && !unbounded) h->mip_x = best_x;
    h->final_status = status;
    h->done = true;
    h->mip = true;
    h->mip_nodes = nodes;
    h->mip_iters = iters;
    *out_status = status;
    return 0;
}

extern "C" int elp_solve(elp_handle* h, int32_t* lp_status) {
    if (!h || !lp_status) return fail(ELP_E_ARG, "elp_solve: NULL argument");
    if (is_group(h)) {
        if (!h->ranks[0]->loaded) return fail(ELP_E_STATE, "elp_solve: no problem loaded");
        std::vector<int32_t> st(h->ranks.size(), 0);
        const int rc = fan_out(h, [&](elp_handle* r, int k) { return elp_solve(r, &st[k]); });
        *lp_status = st[0];
        return rc;
    }
    if (!h->loaded) return fail(ELP_E_STATE, "elp_solve: no problem loaded");
    HIPCHK(hipSetDevice(h->dev));
    const double t0 = now_s();
    int rc;
    if (!h->is_int.empty() && !h->mip && !h->done) {
        rc = run_bnb(h, lp_status);
    } else {
        rc = run_loop(h, INT64_MAX, lp_status);
    }
    h->stats.seconds_total += now_s() - t0;
    return rc;
}

extern "C" int elp_iterate(elp_handle* h, int64_t iters, int32_t* lp_status) {
    if (!h || !lp_status || iters < 0) return fail(ELP_E_ARG, "elp_iterate: bad argument");
    if (is_group(h)) {
        if (!h->ranks[0]->loaded) return fail(ELP_E_STATE, "elp_iterate: no problem loaded");
        std::vector<int32_t> st(h->ranks.size(), 0);
        const int rc = fan_out(h, [&](elp_handle* r, int k) { return elp_iterate(r, iters, &st[k]); });
        *lp_status = st[0];
        return rc;
    }
    if (!h->loaded) return fail(ELP_E_STATE, "elp_iterate: no problem loaded");
    HIPCHK(hipSetDevice(h->dev));
    const double t0 = now_s();
    const int rc = run_loop(h, iters, lp_status);
    h->stats.seconds_total += now_s() - t0;
    return rc;
}

extern "C" int elp_get_solution(elp_handle* h, double* objval, double* x, double* y, int64_t* basis) {
    if (is_group(h) && !h->ranks[0]->loaded) return fail(ELP_E_STATE, "elp_get_solution: no problem loaded");
    if (is_group(h))  // (collective: every rank takes part, rank 0 reports)
        return fan_out(h, [&](elp_handle* r, int k) {
            return k == 0 ? elp_get_solution(r, objval, x, y, basis)
                          : elp_get_solution(r, nullptr, nullptr, nullptr, nullptr);
        });
    if (!h || !h->loaded) return fail(ELP_E_STATE, "elp_get_solution: no problem loaded");
    HIPCHK(hipSetDevice(h->dev));
    const int64_t m = h->m, n = h->n, nl = h->nloc;
    std::vector<double> xs((size_t)n, 0.0);
    if (h->res_fresh && h->res_x.size() == (size_t)n) {
        xs = h->res_x;  // (the resident solver's exit brought them back with the control block)
    } else {
        HIPCHK(hipMemcpyAsync(h->hctl, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
        // structural values: each shard writes its columns into a zeroed full-length
        // vector, the all-reduce (sum with zeros: exact) gives every rank all of x
        double* dx = nullptr;
        HIPCHK(dalloc(&dx, n));
        HIPCHK(hipMemsetAsync(dx, 0, (size_t)n * sizeof(double), h->st));
        HIPCHK(launch_extract(h->d, dx + h->col0, h->st));
        {
            const int rc = h->comm.allreduce_sum_f64(dx, (size_t)n, h->st);
            if (rc) return fail(rc, "solution all-reduce failed");
        }
        HIPCHK(hipMemcpyAsync(xs.data(), dx, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, h->st));
        HIPCHK(hipStreamSynchronize(h->st));
        (void)hipFree(dx);
    }
    (void)nl;
    const DevCtl& c = *h->hctl;
    const double BIG = h->ctl.infinity;
    for (int64_t j = 0; j < n; ++j) xs[j] = unscale_col(h, xs[j], j, 1);  // (exact)
    if (h->mip && !h->mip_x.empty()) xs = h->mip_x;  // branch and bound: the incumbent as found
    const bool unb = h->done && h->final_status == ELP_UNBOUNDED;
    // the unbounded variable's global id (shard-local q -> global)
    const int64_t uvar = unb ? (int64_t)c.unb_var : -1;  // global id
    if (unb && uvar >= 0 && uvar < n) xs[uvar] = c.unb_sig > 0 ? BIG : -BIG;
    if (x) std::memcpy(x, xs.data(), (size_t)n * sizeof(double));
    if (objval) {
        if (unb) {
            *objval = h->maximize ? BIG : -BIG;
        } else {
            // get.objective: sum obj_j x_j (seq fma, the oracle's order)
            double acc = 0.0;
            for (int64_t j = 0; j < n; ++j) {
                acc = std::fma(h->obj_h[j], xs[j], acc);
            }
            *objval = acc;
        }
    }
    if (h->mip) {
        // branch and bound: y and the basis belong to the last node LP, not to
        // the incumbent -- reported as zeros / -1 (include/easylp_hip.h)
        if (y && m) std::fill(y, y + m, 0.0);
        if (basis && m) std::fill(basis, basis + m, (int64_t)-1);
        return 0;
    }
    if (y && m) {
        HIPCHK(hipMemcpyAsync(y, h->d.y, m * sizeof(double), hipMemcpyDeviceToHost, h->st));
        HIPCHK(hipStreamSynchronize(h->st));
        for (int64_t i = 0; i < m; ++i) y[i] = unscale_row(h, h->maximize ? -y[i] : y[i], i, 1);
    }
    if (basis && m) {
        std::vector<int32_t> cover(m), Sl(std::max(c.k, 1));
        HIPCHK(hipMemcpyAsync(cover.data(), h->d.cover, m * sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
        if (c.k)
            HIPCHK(hipMemcpyAsync(Sl.data(), h->d.Sl, c.k * sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
        HIPCHK(hipStreamSynchronize(h->st));
        std::vector<int64_t> bv;
        bv.reserve(m);
        // cover and Sl hold global ids
        for (int64_t i = 0; i < m; ++i)
            if (cover[i] >= 0) bv.push_back(cover[i]);
        for (int p = 0; p < c.k; ++p) bv.push_back(Sl[p]);
        std::sort(bv.begin(), bv.end());
        for (size_t t = 0; t < bv.size() && (int64_t)t < m; ++t) basis[t] = bv[t];
    }
    return 0;
}

// get.sensitivity.obj / get.sensitivity.rhs (R/class.R:613-646) from the final
// basis: the reduced costs and the two MFMA contractions run on the device
// (launch_sensitivity), the per-variable assembly here mirrors
// oracle/elp_oracle.c sensitivity() line by line.
//
// Column-sharded handles (ngpu > 1): every rank runs the same
// launch on its own shard -- reduced costs and the objective-ranging product
// alpha_p. = Minv A[R, shard] over its columns, the rhs ranging (replicated
// A[:, S] Minv) in full -- and the host merges: the interval of a basic
// structural's cost is the intersection of the ranks' intervals (max of the
// lower, min of the upper limits: the same values the single-GPU reduction
// takes, in any order), the per-column entries come from the owning rank.
struct SensPart {
    int64_t col0 = 0, ncols = 0;  // this rank's structurals
    int k = 0;
    std::vector<double> dr, o4, cost, lb, ub, xr, y, b;
    std::vector<int8_t> vs;  // ncols structurals, then m slacks
    std::vector<int32_t> Sl, cover, rpos;
};

static int sens_part(elp_handle* h, SensPart& sp) {
    h->res_fresh = false;
    h->ctl_fresh = false;
    HIPCHK(hipSetDevice(h->dev));
    HIPCHK(hipMemcpyAsync(h->hctl, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    const Dev& d = h->d;
    const int64_t m = h->m, n = d.n;  // (n: this shard's columns)
    const int k = h->hctl->k;
    const int64_t ntc = (n + 63) / 64, ntr = (m + 63) / 64;
    double *dred = nullptr, *TR = nullptr, *plo = nullptr, *phi = nullptr, *qlo = nullptr,
           *qhi = nullptr, *out4 = nullptr;
    auto release = [&]() {
        for (double* p : {dred, TR, plo, phi, qlo, qhi, out4})
            if (p) (void)hipFree(p);
    };
    if (dalloc(&dred, n) != hipSuccess || dalloc(&TR, (size_t)k * n) != hipSuccess ||
        dalloc(&plo, (size_t)k * ntc) != hipSuccess || dalloc(&phi, (size_t)k * ntc) != hipSuccess ||
        dalloc(&qlo, (size_t)k * ntr) != hipSuccess || dalloc(&qhi, (size_t)k * ntr) != hipSuccess ||
        dalloc(&out4, (size_t)4 * k) != hipSuccess) {
        release();
        return fail(ELP_E_NOMEM, "elp_sensitivity: work allocation failed");
    }
    hipError_t e = launch_sensitivity(d, k, dred, TR, plo, phi, qlo, qhi, out4, h->st);
    sp.col0 = h->col0;
    sp.ncols = n;
    sp.k = k;
    sp.dr.resize(n);
    sp.o4.resize(4 * (size_t)k);
    sp.cost.resize(n);
    sp.lb.resize(n);
    sp.ub.resize(n);
    sp.xr.resize(m);
    sp.y.resize(m);
    sp.b.resize(m);
    sp.vs.resize(n + m);
    sp.Sl.resize(k);
    sp.cover.resize(m);
    sp.rpos.resize(m);
    auto d2h = [&](void* dst, const void* src, size_t bytes) {
        if (e == hipSuccess && bytes) e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->st);
    };
    d2h(sp.dr.data(), dred, n * sizeof(double));
    d2h(sp.o4.data(), out4, 4 * (size_t)k * sizeof(double));
    d2h(sp.cost.data(), d.cost, n * sizeof(double));
    d2h(sp.lb.data(), d.lb, n * sizeof(double));
    d2h(sp.ub.data(), d.ub, n * sizeof(double));
    d2h(sp.vs.data(), d.vstat, (n + m) * sizeof(int8_t));
    d2h(sp.Sl.data(), d.Sl, k * sizeof(int32_t));
    d2h(sp.cover.data(), d.cover, m * sizeof(int32_t));
    d2h(sp.rpos.data(), d.rpos, m * sizeof(int32_t));
    d2h(sp.xr.data(), d.xr, m * sizeof(double));
    d2h(sp.y.data(), d.y, m * sizeof(double));
    d2h(sp.b.data(), d.b, m * sizeof(double));
    if (e == hipSuccess) e = hipStreamSynchronize(h->st);
    release();
    if (e != hipSuccess) return fail(ELP_E_HIP, std::string("elp_sensitivity: ") + hipGetErrorString(e));
    return 0;
}

// h: a handle of the solve (rank 0 of a group: scaling, rows, sense are replicated)
static void sens_assemble(const elp_handle* h, const std::vector<SensPart>& parts, double* objfrom,
                          double* objtill, double* duals, double* dualsfrom, double* dualstill) {
    const SensPart& p0 = parts[0];
    const int64_t m = h->m, n = h->n;
    const int k = p0.k;
    const double INF = HUGE_VAL, BIG = h->ctl.infinity;
    auto clip = [&](double v) { return v <= -INF ? -BIG : v >= INF ? BIG : v; };
    const bool mx = h->maximize != 0;
    const double sg = mx ? -1.0 : 1.0;
    // objective-ranging intervals of the basic structurals: intersection over shards
    std::vector<double> olo(p0.o4.begin(), p0.o4.begin() + k), ohi(p0.o4.begin() + k, p0.o4.begin() + 2 * k);
    for (size_t r = 1; r < parts.size(); ++r)
        for (int p = 0; p < k; ++p) {
            olo[p] = std::fmax(olo[p], parts[r].o4[p]);
            ohi[p] = std::fmin(ohi[p], parts[r].o4[k + p]);
        }
    std::vector<int> spos((size_t)n, -1);
    for (int p = 0; p < k; ++p) spos[(size_t)p0.Sl[p]] = p;  // (Sl holds global ids)
    // (the assembly runs on the scaled problem; every output is unscaled)
    if (duals)
        for (int64_t i = 0; i < m; ++i) duals[i] = unscale_row(h, sg * p0.y[i], i, 1);
    for (const SensPart& sp : parts)
        for (int64_t jj = 0; jj < sp.ncols; ++jj) {
            const int64_t j = sp.col0 + jj;
            const double dr = sp.dr[jj];
            if (duals) duals[m + j] = unscale_col(h, sg * dr, j, -1);
            if (!objfrom && !objtill) continue;
            double lo = -INF, hi = INF;
            const double c = sp.cost[jj];
            const int8_t vs = sp.vs[jj];
            if (vs == VS_BASIC) {
                const int p = spos[j];
                lo = c + olo[p];
                hi = c + ohi[p];
            } else if (sp.lb[jj] == sp.ub[jj]) {
            } else if (vs == VS_LOWER) {
                lo = c - dr;
            } else if (vs == VS_UPPER) {
                hi = c - dr;
            } else {
                lo = hi = c;
            }
            if (objfrom) objfrom[j] = clip(unscale_col(h, mx ? -hi : lo, j, -1));
            if (objtill) objtill[j] = clip(unscale_col(h, mx ? -lo : hi, j, -1));
        }
    for (int64_t i = 0; i < m && (dualsfrom || dualstill); ++i) {
        double lo = -INF, hi = INF;
        const double bi = p0.b[i];
        const int u = p0.cover[i];
        if (u == (int)(n + i)) {
            const double act = bi - p0.xr[i];
            if (h->dir_h[i] == ELP_LE) lo = act;
            else if (h->dir_h[i] == ELP_GE) hi = act;
            else lo = hi = bi;
        } else if (u >= (int)(n + m)) {
            lo = hi = bi;
        } else {
            const int c = p0.rpos[i];
            lo = bi + p0.o4[2 * (size_t)k + c];
            hi = bi + p0.o4[3 * (size_t)k + c];
        }
        if (dualsfrom) dualsfrom[i] = clip(unscale_row(h, lo, i, -1));
        if (dualstill) dualstill[i] = clip(unscale_row(h, hi, i, -1));
    }
    for (int64_t j = 0; j < n; ++j) {
        if (dualsfrom) dualsfrom[m + j] = -BIG;
        if (dualstill) dualstill[m + j] = BIG;
    }
}

// One process per GPU (elp_comm_init*): every rank ranged its own columns
// (parts[0]); the ranks' column parts and bump intervals travel in one
// all-gather of fixed-size records -- [col0, ncols, k][o4: 4k][dr, cost, lb, ub,
// status: cap each], cap = ceil(N / P) -- so every rank assembles the full
// report (the replicated rows, y and lists are its own), as an ngpu handle does
// in one process.  A collective: every rank calls elp_sensitivity.
static int sens_gather(elp_handle* h, std::vector<SensPart>& parts) {
    const int P = h->comm.world;
    const int64_t cap = (h->n + P - 1) / P;
    const int k = parts[0].k;
    const size_t R = 3 + 4 * (size_t)k + 5 * (size_t)cap;
    std::vector<double> rec(R, 0.0), all((size_t)P * R);
    {
        const SensPart& sp = parts[0];
        rec[0] = (double)sp.col0;
        rec[1] = (double)sp.ncols;
        rec[2] = (double)sp.k;
        std::copy(sp.o4.begin(), sp.o4.end(), rec.begin() + 3);
        double* c = rec.data() + 3 + 4 * (size_t)k;
        for (int64_t j = 0; j < sp.ncols; ++j) {
            c[j] = sp.dr[(size_t)j];
            c[cap + j] = sp.cost[(size_t)j];
            c[2 * cap + j] = sp.lb[(size_t)j];
            c[3 * cap + j] = sp.ub[(size_t)j];
            c[4 * cap + j] = (double)sp.vs[(size_t)j];
        }
    }
    double *dsend = nullptr, *drecv = nullptr;
    auto release = [&]() {
        if (dsend) (void)hipFree(dsend);
        if (drecv) (void)hipFree(drecv);
    };
    if (dalloc(&dsend, R) != hipSuccess || dalloc(&drecv, (size_t)P * R) != hipSuccess) {
        release();
        return fail(ELP_E_NOMEM, "elp_sensitivity: exchange buffers");
    }
    hipError_t e = hipMemcpyAsync(dsend, rec.data(), R * sizeof(double), hipMemcpyHostToDevice, h->st);
    int rc = e == hipSuccess ? h->comm.allgather(dsend, drecv, R * sizeof(double), h->st) : 0;
    if (e == hipSuccess && !rc)
        e = hipMemcpyAsync(all.data(), drecv, (size_t)P * R * sizeof(double), hipMemcpyDeviceToHost, h->st);
    if (e == hipSuccess && !rc) e = hipStreamSynchronize(h->st);
    release();
    if (rc) return fail(rc, "elp_sensitivity: the ranks' report all-gather failed");
    if (e != hipSuccess) return fail(ELP_E_HIP, std::string("elp_sensitivity: ") + hipGetErrorString(e));
    SensPart mine = std::move(parts[0]);  // (the replicated fields come from this rank)
    parts.assign((size_t)P, SensPart{});
    for (int r = 0; r < P; ++r) {
        const double* x = all.data() + (size_t)r * R;
        SensPart& sp = parts[(size_t)r];
        sp.col0 = (int64_t)x[0];
        sp.ncols = (int64_t)x[1];
        sp.k = (int)x[2];
        if (sp.ncols < 0) return fail(ELP_E_STATE, "elp_sensitivity: rank " + std::to_string(r) + " failed its part");
        if (sp.k != k || sp.ncols > cap) return fail(ELP_E_STATE, "elp_sensitivity: the ranks' bases differ");
        sp.o4.assign(x + 3, x + 3 + 4 * (size_t)k);
        const double* c = x + 3 + 4 * (size_t)k;
        sp.dr.assign(c, c + sp.ncols);
        sp.cost.assign(c + cap, c + cap + sp.ncols);
        sp.lb.assign(c + 2 * cap, c + 2 * cap + sp.ncols);
        sp.ub.assign(c + 3 * cap, c + 3 * cap + sp.ncols);
        sp.vs.resize((size_t)sp.ncols);
        for (int64_t j = 0; j < sp.ncols; ++j) sp.vs[(size_t)j] = (int8_t)c[4 * cap + j];
    }
    // rank 0's slot carries the replicated rows / duals / lists (identical everywhere)
    SensPart& p0 = parts[0];
    p0.xr = std::move(mine.xr);
    p0.y = std::move(mine.y);
    p0.b = std::move(mine.b);
    p0.Sl = std::move(mine.Sl);
    p0.cover = std::move(mine.cover);
    p0.rpos = std::move(mine.rpos);
    return 0;
}

// the state checks of a rank handle (every rank of a group holds the same)
static int sens_check(elp_handle* h) {
    if (!h || !h->loaded) return fail(ELP_E_STATE, "elp_sensitivity: no problem loaded");
    if (!h->done || h->final_status != ELP_OPTIMAL)
        return fail(ELP_E_STATE, "elp_sensitivity: problem is not optimal");
    if (h->mip || !h->is_int.empty())  // R/class.R:617-618, :634-635
        return fail(ELP_E_STATE, "Sensitivity unavailable for problems with integer/binary variables");
    return 0;
}

extern "C" int elp_sensitivity(elp_handle* h, double* objfrom, double* objtill, double* duals,
                               double* dualsfrom, double* dualstill) {
    if (is_group(h)) {
        // (no collective: the ranks' reports meet in this process's memory)
        for (elp_handle* r : h->ranks) {
            const int rc = sens_check(r);
            if (rc) return rc;
        }
        std::vector<SensPart> parts(h->ranks.size());
        const int rc = fan_out(h, [&](elp_handle* r, int k) { return sens_part(r, parts[(size_t)k]); }, false);
        if (rc) return rc;
        sens_assemble(h->ranks[0], parts, objfrom, objtill, duals, dualsfrom, dualstill);
        return 0;
    }
    const int rc0 = sens_check(h);
    if (rc0) return rc0;
    std::vector<SensPart> parts(1);
    const int rc = sens_part(h, parts[0]);
    if (h->comm.kind != 0) {
        // a collective: a rank whose part failed still joins the all-gather,
        // its record flagged (ncols = -1), so every rank fails together and no
        // peer waits for it; the record size follows the replicated k
        const std::string err = g_err;
        if (rc) {
            parts[0] = SensPart{};
            parts[0].k = h->hctl ? h->hctl->k : 0;
            parts[0].ncols = -1;
        }
        const int rg = sens_gather(h, parts);
        if (rc) return fail(rc, err);
        if (rg) return rg;
    } else if (rc) {
        return rc;
    }
    sens_assemble(h, parts, objfrom, objtill, duals, dualsfrom, dualstill);
    return 0;
}

extern "C" int elp_get_stats(elp_handle* h, elp_stats* st) {
    if (is_group(h)) return elp_get_stats(h->ranks[0], st);
    if (!h || !st) return fail(ELP_E_ARG, "elp_get_stats: NULL argument");
    if (h->loaded) {
        HIPCHK(hipSetDevice(h->dev));
        if (!h->res_fresh) {
            HIPCHK(hipMemcpyAsync(h->hctl, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
            HIPCHK(hipStreamSynchronize(h->st));
        }
        const DevCtl& c = *h->hctl;
        h->stats.iterations = c.iter;
        h->stats.phase1_iterations = c.phase1_iters;
        h->stats.bound_flips = c.flips;
        h->stats.degenerate = c.degenerate;
        h->stats.bump_dim = c.k;
        h->stats.y_rows = c.ny;
        h->stats.mip_nodes = h->mip ? h->mip_nodes : 0;
        h->stats.mip_lp_iterations = h->mip ? h->mip_iters : 0;
        h->stats.price_bytes = c.price_bytes;
        h->stats.iter_bytes = c.iter_bytes;
        h->stats.exchange_rtt_us = h->comm.p2p ? h->comm.rtt_us : 0.0;
        h->stats.dual_iterations = c.dual_iters;
        h->stats.simplex = h->dual_used ? ELP_SIMPLEX_DUAL_PRIMAL : ELP_SIMPLEX_PRIMAL_PRIMAL;
        if (h->d.ptimer) {
            h->stats.price_seconds = 1e-8 * (double)c.price_ticks;
            h->stats.price_timed_launches = c.price_timed;
            h->stats.price_timed_bytes = c.price_tbytes;
        }
    }
    *st = h->stats;
    return 0;
}

extern "C" int elp_set_trace(elp_handle* h, int64_t capacity) {
    if (is_group(h) && capacity >= 0)
        return fan_out(h, [&](elp_handle* r, int) { return elp_set_trace(r, capacity); }, false);
    if (!h || capacity < 0) return fail(ELP_E_ARG, "elp_set_trace: bad argument");
    if (h->loaded) return fail(ELP_E_STATE, "elp_set_trace: call before elp_load_*");
    h->trace_cap = capacity;
    return 0;
}

extern "C" int elp_get_trace(elp_handle* h, int64_t* pairs, int64_t capacity, int64_t* count) {
    if (is_group(h)) return elp_get_trace(h->ranks[0], pairs, capacity, count);
    if (!h || !count) return fail(ELP_E_ARG, "elp_get_trace: NULL argument");
    if (!h->loaded) return fail(ELP_E_STATE, "elp_get_trace: no problem loaded");
    HIPCHK(hipSetDevice(h->dev));
    HIPCHK(hipMemcpyAsync(h->hctl, h->d.ctl, sizeof(DevCtl), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    const int64_t cnt = std::min<int64_t>(std::min<int64_t>(h->hctl->iter, h->trace_cap), capacity);
    if (cnt > 0 && pairs) {
        HIPCHK(hipMemcpyAsync(pairs, h->d.trace, 2 * cnt * sizeof(int64_t), hipMemcpyDeviceToHost, h->st));
        HIPCHK(hipStreamSynchronize(h->st));
    }
    *count = cnt;
    return 0;
}

extern "C" void elp_destroy(elp_handle* h) {
    if (h && h->stamp_n) {
        std::fprintf(stderr, "k_ratio stamps (us after workgroup 0's start; ELP_STAMPS=2: the first workgroup's; %lld iterations):",
                     (long long)h->stamp_n);
        const char* nm[11] = {"wg0", "ctl", "pass1", "decide", "binv", "dual", "book", "end", "last_start",
                              "main_end", "ar_end"};
        for (int i = 0; i < 11; ++i) std::fprintf(stderr, " %s=%.2f", nm[i], h->stamp_sum[i] / h->stamp_n / 1e3);
        std::fprintf(stderr, "\nk_select_ftran stamps (us after its workgroup 0 starts): ctl=%.2f decide=%.2f end=%.2f\n",
                     h->stamp_sum[13] / h->stamp_n / 1e3, h->stamp_sum[14] / h->stamp_n / 1e3,
                     h->stamp_sum[15] / h->stamp_n / 1e3);
        std::fprintf(stderr, "k_ftran_zr stamps (us after its workgroup 0 starts): ctl=%.2f z=%.2f emitted=%.2f\n",
                     h->stamp_sum[17] / h->stamp_n / 1e3, h->stamp_sum[18] / h->stamp_n / 1e3,
                     h->stamp_sum[19] / h->stamp_n / 1e3);
        std::fprintf(stderr, "k_dual_bfrt stamps (us after its start): compacted=%.2f decided=%.2f end=%.2f\n",
                     h->stamp_sum[21] / h->stamp_n / 1e3, h->stamp_sum[22] / h->stamp_n / 1e3,
                     h->stamp_sum[23] / h->stamp_n / 1e3);
        std::fprintf(stderr, "k_dual_bfrt counts (per iteration): candidates=%.1f flips=%.2f one_wave=%.3f rounds=%.2f "
                     "(wave: loaded=%.2f us)\n",
                     h->stamp_sum[24] / h->stamp_n, h->stamp_sum[25] / h->stamp_n, h->stamp_sum[26] / h->stamp_n,
                     h->stamp_sum[28] / h->stamp_n, h->stamp_sum[27] / std::max(1.0, h->stamp_sum[34]) / 1e3);
        if (h->stamp_sum[38] > 0)
            std::fprintf(stderr, "k_dual_bfrt shader clock (s_memtime over s_memrealtime): %.0f MHz\n",
                         1e3 * h->stamp_sum[37] / h->stamp_sum[38]);
        const double nt = std::max(1.0, h->stamp_sum[36]);
        std::fprintf(stderr, "k_dual_bfrt fast tail (us after its start; rounds over %.0f launches, the a_F phases over "
                     "the %.0f with flips): rounds done %.2f, a_F offsets %.2f, chains %.2f, support scan %.2f, "
                     "a_F[R] list %.2f\n",
                     h->stamp_sum[35], h->stamp_sum[36], h->stamp_sum[29] / std::max(1.0, h->stamp_sum[35]) / 1e3,
                     h->stamp_sum[30] / nt / 1e3, h->stamp_sum[31] / nt / 1e3, h->stamp_sum[32] / nt / 1e3,
                     h->stamp_sum[33] / nt / 1e3);
        const double nf = std::max(1.0, h->stamp_sum[48]);
        std::fprintf(stderr, "k_dual_bfrt with a fast tail (%.0f launches; us after its start): compacted %.2f, "
                     "records loaded %.2f, rounds done %.2f, decided %.2f, tail start %.2f, end %.2f "
                     "(candidates %.1f, rounds %.2f)\n",
                     h->stamp_sum[48], h->stamp_sum[40] / nf / 1e3, h->stamp_sum[41] / nf / 1e3,
                     h->stamp_sum[42] / nf / 1e3, h->stamp_sum[43] / nf / 1e3, h->stamp_sum[44] / nf / 1e3,
                     h->stamp_sum[45] / nf / 1e3, h->stamp_sum[46] / nf, h->stamp_sum[47] / nf);
        for (int q = 0; q < 3; ++q) {
            const double* b = &h->stamp_sum[49 + 3 * q];
            std::fprintf(stderr, "k_dual_bfrt a_F by %s: %.0f launches, end %.2f us, flip entries %.1f\n",
                         q == 0 ? "one wave" : q == 1 ? "LDS block" : "column walk", b[0],
                         b[1] / std::max(1.0, b[0]) / 1e3, b[2] / std::max(1.0, b[0]));
        }
    }
    if (!h) return;
    destroy_group(h);
    (void)hipSetDevice(h->dev);
    if (h->st) (void)hipStreamSynchronize(h->st);
    if (getenv("ELP_DEBUG_ENQUEUE"))
        fprintf(stderr, "elp: host enqueue %.4f s, poll wait %.4f s, polls %lld\n", h->dbg_enqueue,
                h->dbg_wait, (long long)h->stats.host_polls);
    // a plain one-GPU handle leaves its resources for the next elp_create (Spare)
    if (h->st && spares_on() && h->ranks.empty() && h->comm.kind == 0 && h->ctl.ngpu <= 1 && h->ev.empty()) {
        free_dev(h, true);  // (every buffer into the pool, A's copy kept)
        Spare sp;
        sp.dev = h->dev;
        sp.st = h->st;
        sp.pool = std::move(h->pool);
        for (auto& kv : sp.pool) sp.bytes += kv.first;
        sp.keep_A = h->keep_A;
        sp.keep_A_bytes = h->keep_A_bytes;
        sp.bytes += sp.keep_A_bytes;
        sp.hctl = h->hctl;
        sp.resout = h->d_resout;
        sp.resx_n = h->n;
        sp.respin = h->res_pin;
        h->pool.clear();
        h->keep_A = nullptr;
        h->hctl = nullptr;
        h->d_resout = nullptr;
        h->d_resx = nullptr;
        h->res_pin = nullptr;
        h->st = nullptr;
        std::vector<Spare> drop;
        {
            std::lock_guard<std::mutex> lk(g_spare_mu);
            size_t tot = sp.bytes;
            for (const Spare& o : g_spares) tot += o.bytes;
            if (sp.bytes <= SPARE_BYTES) {
                g_spares.push_back(std::move(sp));
                while (!g_spares.empty() && ((int)g_spares.size() > SPARE_MAX || tot > SPARE_BYTES)) {
                    tot -= g_spares.front().bytes;  // (the oldest goes)
                    drop.push_back(std::move(g_spares.front()));
                    g_spares.erase(g_spares.begin());
                }
            } else {
                drop.push_back(std::move(sp));
            }
        }
        for (Spare& o : drop) spare_free(o);
        (void)hipSetDevice(h->dev);
    }
    free_dev(h);
    release_kept(h);
    if (h->d_resout) (void)hipFree(h->d_resout);
    if (h->res_pin) (void)hipHostFree(h->res_pin);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    h->comm.destroy();
    if (h->st) (void)hipStreamDestroy(h->st);
    delete h;
}

extern "C" int elp_comm_unique_id(uint8_t id[128]) { return elp::Comm::unique_id(id); }

extern "C" int elp_comm_init(elp_handle* h, const uint8_t id[128], int32_t world_size, int32_t rank) {
    if (is_group(h)) return fail(ELP_E_STATE, "an ngpu > 1 handle owns its communicator");
    if (!h || !id || world_size < 1 || rank < 0 || rank >= world_size)
        return fail(ELP_E_ARG, "elp_comm_init: bad argument");
    if (h->loaded) return fail(ELP_E_STATE, "elp_comm_init: call before elp_load_*");
    HIPCHK(hipSetDevice(h->dev));
    const int rc = h->comm.init_rccl(id, world_size, rank);
    return rc ? fail(rc, "RCCL communicator init failed") : 0;
}

extern "C" int elp_comm_enable_p2p(elp_handle* h) {
    if (is_group(h)) return fail(ELP_E_STATE, "an ngpu > 1 handle owns its communicator");
    if (!h) return fail(ELP_E_ARG, "elp_comm_enable_p2p: NULL handle");
    if (h->loaded) return fail(ELP_E_STATE, "elp_comm_enable_p2p: call before elp_load_*");
    if (h->comm.kind == 0) return 0;  // one rank: nothing to exchange
    if (h->comm.world > 64) return fail(ELP_E_UNSUPPORTED, "elp_comm_enable_p2p: more than 64 ranks");
    HIPCHK(hipSetDevice(h->dev));
    const int rc = h->comm.enable_p2p(sizeof(MboxRec), h->st, h->ctl.mailbox_timeout);
    return rc ? fail(rc, "elp_comm_enable_p2p: mailbox allocation / IPC exchange failed") : 0;
}

extern "C" int elp_comm_init_host(elp_handle* h, int32_t world_size, int32_t rank,
                                  elp_host_allgather_fn ag, elp_host_allreduce_fn ar,
                                  elp_host_bcast_fn bc, void* user) {
    if (is_group(h)) return fail(ELP_E_STATE, "an ngpu > 1 handle owns its communicator");
    if (!h || world_size < 1 || rank < 0 || rank >= world_size)
        return fail(ELP_E_ARG, "elp_comm_init_host: bad argument");
    if (h->loaded) return fail(ELP_E_STATE, "elp_comm_init_host: call before elp_load_*");
    const int rc = h->comm.init_host(world_size, rank, ag, ar, bc, user);
    return rc ? fail(rc, "elp_comm_init_host: NULL transport") : 0;
}
