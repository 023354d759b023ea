// elp_comm.hip -- RCCL and host-callback transports for the sharded solve.
#include "elp_comm.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace elp {

int Comm::unique_id(uint8_t id[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return ELP_E_COMM;
    std::memcpy(id, &u, 128);
    return 0;
}

int Comm::init_rccl(const uint8_t id[128], int world_size, int rank_) {
    world = world_size;
    rank = rank_;
    // one rank: plain single-GPU path, unless ELP_RCCL_SINGLE=1 asks for the
    // sharded pipeline over a 1-rank RCCL communicator (tests on one GPU)
    if (world == 1 && !std::getenv("ELP_RCCL_SINGLE")) {
        kind = 0;
        return 0;
    }
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    if (!scratch && hipMalloc(&scratch, SCRATCH_BYTES) != hipSuccess) {
        scratch = nullptr;
        return ELP_E_NOMEM;
    }
    ncclComm_t c = nullptr;
    if (ncclCommInitRank(&c, world, u, rank) != ncclSuccess) return ELP_E_COMM;
    nccl = c;
    kind = 1;
    return 0;
}

int Comm::adopt_rccl(void* comm, int world_size, int rank_) {
    world = world_size;
    rank = rank_;
    if (!scratch && hipMalloc(&scratch, SCRATCH_BYTES) != hipSuccess) {
        scratch = nullptr;
        return ELP_E_NOMEM;
    }
    nccl = comm;
    kind = 1;
    return 0;
}

int Comm::init_all(std::vector<void*>& comms, const std::vector<int>& devs) {
    std::vector<ncclComm_t> c(devs.size(), nullptr);
    if (ncclCommInitAll(c.data(), (int)devs.size(), devs.data()) != ncclSuccess) return ELP_E_COMM;
    comms.assign(c.begin(), c.end());
    return 0;
}

// ---------------------------------------------------------------- threads
bool ThreadGroup::barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return false;
    const uint64_t my = gen;
    if (++arrived == world) {
        arrived = 0;
        ++gen;
        cv.notify_all();
        return true;
    }
    cv.wait(lk, [&] { return gen != my || aborted; });
    return !aborted || gen != my;
}

void ThreadGroup::abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
}

void ThreadGroup::reset() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = false;
    arrived = 0;
}

// every collective: (rank 0 sizes the area) barrier, deposit, barrier, read,
// barrier -- the last one keeps the area intact until every rank has read it
int ThreadGroup::allgather(const void* send, void* recv, size_t bytes, void* user) {
    ThreadRank* tr = static_cast<ThreadRank*>(user);
    ThreadGroup& g = *tr->g;
    if (!g.barrier()) return 1;
    if (tr->rank == 0) g.buf.resize(bytes * (size_t)g.world);
    if (!g.barrier()) return 1;
    std::memcpy(g.buf.data() + bytes * (size_t)tr->rank, send, bytes);
    if (!g.barrier()) return 1;
    std::memcpy(recv, g.buf.data(), bytes * (size_t)g.world);
    return g.barrier() ? 0 : 1;
}

int ThreadGroup::allreduce(void* buf, size_t count, int32_t dtype, void* user) {
    ThreadRank* tr = static_cast<ThreadRank*>(user);
    ThreadGroup& g = *tr->g;
    const size_t es = dtype == 0 ? sizeof(double) : sizeof(int32_t);
    const size_t bytes = count * es;
    if (!g.barrier()) return 1;
    if (tr->rank == 0) g.buf.resize(bytes * (size_t)g.world);
    if (!g.barrier()) return 1;
    std::memcpy(g.buf.data() + bytes * (size_t)tr->rank, buf, bytes);
    if (!g.barrier()) return 1;
    if (dtype == 0) {  // f64 sum in rank order
        double* out = static_cast<double*>(buf);
        const double* all = reinterpret_cast<const double*>(g.buf.data());
        for (size_t i = 0; i < count; ++i) {
            double acc = all[i];
            for (int r = 1; r < g.world; ++r) acc = acc + all[(size_t)r * count + i];
            out[i] = acc;
        }
    } else {  // i32 max
        int32_t* out = static_cast<int32_t*>(buf);
        const int32_t* all = reinterpret_cast<const int32_t*>(g.buf.data());
        for (size_t i = 0; i < count; ++i) {
            int32_t v = all[i];
            for (int r = 1; r < g.world; ++r) v = std::max(v, all[(size_t)r * count + i]);
            out[i] = v;
        }
    }
    return g.barrier() ? 0 : 1;
}

int ThreadGroup::bcast(void* buf, size_t bytes, int32_t root, void* user) {
    ThreadRank* tr = static_cast<ThreadRank*>(user);
    ThreadGroup& g = *tr->g;
    if (!g.barrier()) return 1;
    if (tr->rank == root) g.buf.assign(static_cast<unsigned char*>(buf), static_cast<unsigned char*>(buf) + bytes);
    if (!g.barrier()) return 1;
    if (tr->rank != root) std::memcpy(buf, g.buf.data(), bytes);
    return g.barrier() ? 0 : 1;
}

int Comm::init_host(int world_size, int rank_, elp_host_allgather_fn ag, elp_host_allreduce_fn ar,
                    elp_host_bcast_fn bc, void* user) {
    if (!ag || !ar || !bc) return ELP_E_ARG;
    world = world_size;
    rank = rank_;
    kind = world > 1 ? 2 : 0;
    if (!scratch && hipMalloc(&scratch, SCRATCH_BYTES) != hipSuccess) {
        scratch = nullptr;
        return ELP_E_NOMEM;
    }
    h_allgather = ag;
    h_allreduce = ar;
    h_bcast = bc;
    h_user = user;
    return 0;
}

// Round-trip probe of freshly mapped mailboxes: thread t stores a reserved
// sequence word into this rank's slots (both parities) of rank t's mailbox,
// then waits (the mailbox timeout at most) for rank t's word in its own.  Proves, before the
// first solve, that remote stores land and become visible to the polling
// loads (p2p_exchange's protocol); the reserved words can never equal a real
// iteration's sequence (epoch << 40 | iteration + 1).  Then MBOX_ROUNDS
// exchange rounds of the solver's shape (store this round's word into every
// peer's slot of the round's parity, wait for every peer's): ok_out[1] = the
// 100 MHz ticks they took on thread 0, i.e. the per-iteration cost of the
// exchange with every kernel already running.
constexpr int64_t MBOX_PROBE_SEQ = INT64_MAX;
constexpr int MBOX_ROUNDS = 64;
__global__ void k_mbox_probe(void* const* peers, void* mine, int P, int rank, int64_t rec, int* ok_out,
                             unsigned long long ticks) {
    __shared__ int fail;
    const int t = threadIdx.x;
    if (t == 0) fail = 0;
    __syncthreads();
    auto slot = [&](void* base, int par, int r) {
        return reinterpret_cast<int64_t*>(static_cast<char*>(base) + (par * P + r) * rec + rec - 8);
    };
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    auto wait_for = [&](int64_t* s, int64_t want) {
        while (__hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != want) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {  // 100 MHz clock
                atomicOr(&fail, 1);
                return;
            }
        }
    };
    if (t < P) {
        __threadfence_system();
        for (int par = 0; par < 2; ++par)
            __hip_atomic_store(slot(peers[t], par, rank), MBOX_PROBE_SEQ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
    if (t < P)
        for (int par = 0; par < 2; ++par) wait_for(slot(mine, par, t), MBOX_PROBE_SEQ);
    __syncthreads();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 1; r <= MBOX_ROUNDS && !fail; ++r) {
        const int par = r & 1;
        const int64_t want = MBOX_PROBE_SEQ - r;
        if (t < P) {
            __threadfence_system();
            __hip_atomic_store(slot(peers[t], par, rank), want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            wait_for(slot(mine, par, t), want);
        }
        __syncthreads();
    }
    if (t == 0) {
        ok_out[0] = fail ? 0 : 1;
        ok_out[1] = fail ? 0 : (int)(__builtin_amdgcn_s_memrealtime() - r0);
    }
}

hipError_t launch_mbox_probe(void* const* dpeers, void* mine, int P, int rank, int64_t rec_bytes, int32_t* ok,
                             unsigned long long ticks, hipStream_t st) {
    hipLaunchKernelGGL(k_mbox_probe, dim3(1), dim3(64), 0, st, dpeers, mine, P, rank, rec_bytes, ok, ticks);
    return hipGetLastError();
}

double mbox_rtt_us(int32_t ticks) { return ticks > 0 ? 10.0 * 1e-3 * (double)ticks / MBOX_ROUNDS : 0.0; }

void Comm::adopt_p2p(void* mine, void** dpeers_dev) {
    mbox = mine;
    dpeers = dpeers_dev;
    p2p = 1;
}

void Comm::abort_rccl() {
    bool expect = false;
    if (kind == 1 && nccl && aborted.compare_exchange_strong(expect, true)) (void)ncclCommAbort((ncclComm_t)nccl);
}

// Collective over the communicator: every rank takes every step (the handle
// all-gather and the final agreement), so a rank that fails to allocate or to
// map a peer does not strand the others; if any rank failed, none uses p2p.
int Comm::enable_p2p(size_t rec_bytes, hipStream_t st, double timeout_s) {
    if (kind == 0) return ELP_E_STATE;
    if (p2p) return 0;
    // staging of the two collectives below: the scratch buffer allocated with
    // the communicator, so no allocation here can make this rank skip them
    // (checked before anything is allocated: callers keep world <= 64)
    if (!scratch || world > SCRATCH_RANKS) return ELP_E_STATE;
    const size_t bytes = 2 * (size_t)world * rec_bytes;
    int ok = 1;
    hipIpcMemHandle_t mine;
    std::memset(&mine, 0, sizeof(mine));
    // uncached: a peer's remote store and this rank's polling load meet in memory
    if (hipExtMallocWithFlags(&mbox, bytes, hipDeviceMallocUncached) != hipSuccess) {
        mbox = nullptr;
        ok = 0;
    }
    if (ok && hipMemset(mbox, 0, bytes) != hipSuccess) ok = 0;
    if (ok && hipIpcGetMemHandle(&mine, mbox) != hipSuccess) ok = 0;
    static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
    unsigned char* dstage = static_cast<unsigned char*>(scratch);
    std::vector<unsigned char> all(64 * (size_t)world);
    int rc = hipMemcpy(dstage + 64 * world, &mine, 64, hipMemcpyHostToDevice) == hipSuccess ? 0 : ELP_E_HIP;
    if (!rc) rc = allgather(dstage + 64 * world, dstage, 64, st);
    if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = ELP_E_HIP;
    if (!rc && hipMemcpy(all.data(), dstage, all.size(), hipMemcpyDeviceToHost) != hipSuccess) rc = ELP_E_HIP;
    std::vector<void*> ptrs((size_t)world, nullptr);
    for (int r = 0; !rc && ok && r < world; ++r) {
        if (r == rank) {
            ptrs[r] = mbox;
            continue;
        }
        hipIpcMemHandle_t hd;
        std::memcpy(&hd, all.data() + 64 * (size_t)r, 64);
        if (hipIpcOpenMemHandle(&ptrs[r], hd, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            ok = 0;
            break;
        }
        opened.push_back(ptrs[r]);
    }
    if (!rc && ok) {
        if (hipMalloc((void**)&dpeers, sizeof(void*) * (size_t)world) != hipSuccess) ok = 0;
        else if (hipMemcpy(dpeers, ptrs.data(), sizeof(void*) * (size_t)world, hipMemcpyHostToDevice) != hipSuccess)
            ok = 0;
    }
    // every rank that mapped all peers probes the round trip (a rank that did
    // not leaves its peers' probes to time out: they fail the agreement too)
    if (!rc && ok) {
        int32_t* dok = reinterpret_cast<int32_t*>(dstage);
        int32_t hok[2] = {0, 0};
        const double secs = timeout_s > 0 ? timeout_s : 2.0;
        if (launch_mbox_probe((void* const*)dpeers, mbox, world, rank, (int64_t)rec_bytes, dok,
                              (unsigned long long)(secs * 1e8), st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess ||
            hipMemcpy(hok, dok, sizeof(hok), hipMemcpyDeviceToHost) != hipSuccess || !hok[0])
            ok = 0;
        else
            rtt_us = mbox_rtt_us(hok[1]);
    }
    // agreement: max over ranks of "failed"
    int32_t failed = rc || !ok;
    int32_t* dflag = reinterpret_cast<int32_t*>(dstage + 64 * ((size_t)world + 1));
    if (!rc && hipMemcpy(dflag, &failed, sizeof(failed), hipMemcpyHostToDevice) != hipSuccess) rc = ELP_E_HIP;
    if (!rc) rc = allreduce_max_i32(dflag, 1, st);
    if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = ELP_E_HIP;
    if (!rc && hipMemcpy(&failed, dflag, sizeof(failed), hipMemcpyDeviceToHost) != hipSuccess) rc = ELP_E_HIP;
    if (rc || failed) {
        for (void* p : opened) (void)hipIpcCloseMemHandle(p);
        opened.clear();
        if (dpeers) (void)hipFree(dpeers);
        if (mbox) (void)hipFree(mbox);
        dpeers = nullptr;
        mbox = nullptr;
        return rc ? rc : ELP_E_COMM;
    }
    p2p = 1;
    return 0;
}

void Comm::destroy() {
    for (void* p : opened) (void)hipIpcCloseMemHandle(p);
    opened.clear();
    if (dpeers) (void)hipFree(dpeers);
    if (mbox) (void)hipFree(mbox);
    dpeers = nullptr;
    mbox = nullptr;
    p2p = 0;
    if (kind == 1 && nccl && !aborted) ncclCommDestroy((ncclComm_t)nccl);
    aborted = false;
    if (scratch) (void)hipFree(scratch);
    scratch = nullptr;
    nccl = nullptr;
    kind = 0;
    world = 1;
}

int Comm::allgather(const void* dsend, void* drecv, size_t bytes, hipStream_t st) {
    if (aborted) return ELP_E_COMM;
    if (kind == 0) {
        if (dsend != drecv && hipMemcpyAsync(drecv, dsend, bytes, hipMemcpyDeviceToDevice, st) != hipSuccess)
            return ELP_E_HIP;
        return 0;
    }
    if (kind == 1)
        return ncclAllGather(dsend, drecv, bytes, ncclUint8, (ncclComm_t)nccl, st) == ncclSuccess ? 0 : ELP_E_COMM;
    stage.resize(bytes * (world + 1));
    unsigned char* snd = stage.data() + bytes * world;
    if (hipMemcpyAsync(snd, dsend, bytes, hipMemcpyDeviceToHost, st) != hipSuccess) return ELP_E_HIP;
    if (hipStreamSynchronize(st) != hipSuccess) return ELP_E_HIP;
    if (h_allgather(snd, stage.data(), bytes, h_user) != 0) return ELP_E_COMM;
    if (hipMemcpyAsync(drecv, stage.data(), bytes * world, hipMemcpyHostToDevice, st) != hipSuccess) return ELP_E_HIP;
    return hipStreamSynchronize(st) == hipSuccess ? 0 : ELP_E_HIP;
}

static int host_allreduce(Comm& c, void* dbuf, size_t count, size_t esize, int dtype, hipStream_t st) {
    const size_t bytes = count * esize;
    c.stage.resize(bytes);
    if (hipMemcpyAsync(c.stage.data(), dbuf, bytes, hipMemcpyDeviceToHost, st) != hipSuccess) return ELP_E_HIP;
    if (hipStreamSynchronize(st) != hipSuccess) return ELP_E_HIP;
    if (c.h_allreduce(c.stage.data(), count, dtype, c.h_user) != 0) return ELP_E_COMM;
    if (hipMemcpyAsync(dbuf, c.stage.data(), bytes, hipMemcpyHostToDevice, st) != hipSuccess) return ELP_E_HIP;
    return hipStreamSynchronize(st) == hipSuccess ? 0 : ELP_E_HIP;
}

int Comm::allreduce_sum_f64(double* dbuf, size_t count, hipStream_t st) {
    if (aborted) return ELP_E_COMM;
    if (kind == 0) return 0;
    if (kind == 1)
        return ncclAllReduce(dbuf, dbuf, count, ncclFloat64, ncclSum, (ncclComm_t)nccl, st) == ncclSuccess
                   ? 0 : ELP_E_COMM;
    return host_allreduce(*this, dbuf, count, sizeof(double), 0, st);
}

int Comm::allreduce_max_i32(int32_t* dbuf, size_t count, hipStream_t st) {
    if (aborted) return ELP_E_COMM;
    if (kind == 0) return 0;
    if (kind == 1)
        return ncclAllReduce(dbuf, dbuf, count, ncclInt32, ncclMax, (ncclComm_t)nccl, st) == ncclSuccess
                   ? 0 : ELP_E_COMM;
    return host_allreduce(*this, dbuf, count, sizeof(int32_t), 1, st);
}

int Comm::bcast_f64(double* dbuf, size_t count, int root, hipStream_t st) {
    if (aborted) return ELP_E_COMM;
    if (kind == 0) return 0;
    if (kind == 1)
        return ncclBroadcast(dbuf, dbuf, count, ncclFloat64, root, (ncclComm_t)nccl, st) == ncclSuccess
                   ? 0 : ELP_E_COMM;
    const size_t bytes = count * sizeof(double);
    stage.resize(bytes);
    if (hipMemcpyAsync(stage.data(), dbuf, bytes, hipMemcpyDeviceToHost, st) != hipSuccess) return ELP_E_HIP;
    if (hipStreamSynchronize(st) != hipSuccess) return ELP_E_HIP;
    if (h_bcast(stage.data(), bytes, root, h_user) != 0) return ELP_E_COMM;
    if (hipMemcpyAsync(dbuf, stage.data(), bytes, hipMemcpyHostToDevice, st) != hipSuccess) return ELP_E_HIP;
    return hipStreamSynchronize(st) == hipSuccess ? 0 : ELP_E_HIP;
}

}  // namespace elp
