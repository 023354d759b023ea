// elp_comm.h -- communicator for the column-sharded solve.
//
// Three primitives, all on device buffers and ordered on the solver stream:
// all-gather of fixed-size records, all-reduce (f64 sum / i32 max) and
// broadcast.  Transports: RCCL (one process per GPU, over xGMI), or host
// callbacks (the caller moves host copies, e.g. with torch.distributed gloo;
// used to run several ranks on one GPU in tests).  World size 1 is a no-op.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "../../include/easylp_hip.h"

namespace elp {

// In-process transport of a single-process multi-device handle
// (elp_control.ngpu) whose ranks share a device: the ranks are host threads of
// one process and exchange host copies through a shared staging area, a
// generation-counted barrier between the phases of each collective.  The
// reductions run in rank order on every rank, so all ranks hold identical
// bits.  abort() releases every waiting rank (their collectives fail).
struct ThreadGroup {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool aborted = false;
    std::vector<unsigned char> buf;
    explicit ThreadGroup(int P) : world(P) {}
    bool barrier();
    void abort();
    void reset();
    // elp_host_*_fn callbacks; user = &ranks[r] (a ThreadRank)
    static int allgather(const void* send, void* recv, size_t bytes, void* user);
    static int allreduce(void* buf, size_t count, int32_t dtype, void* user);
    static int bcast(void* buf, size_t bytes, int32_t root, void* user);
};
struct ThreadRank {
    ThreadGroup* g;
    int rank;
};

struct Comm {
    int world = 1, rank = 0;
    int kind = 0;          // 0 none, 1 rccl, 2 host callbacks
    void* nccl = nullptr;  // ncclComm_t
    elp_host_allgather_fn h_allgather = nullptr;
    elp_host_allreduce_fn h_allreduce = nullptr;
    elp_host_bcast_fn h_bcast = nullptr;
    void* h_user = nullptr;
    std::vector<unsigned char> stage;  // host staging for the callback transport
    // xGMI mailbox (enable_p2p): every iteration each rank writes its min-loc
    // record straight into every peer's mailbox (2 parities x world records,
    // uncached device memory shared by IPC) -- no collective launch per iteration
    void* mbox = nullptr;              // this rank's mailbox
    void** dpeers = nullptr;           // device array: every rank's mailbox, mapped here
    std::vector<void*> opened;         // IPC-opened peer mailboxes
    int p2p = 0;
    // device scratch for setup collectives (enable_p2p), allocated at init
    static constexpr int SCRATCH_RANKS = 64;
    static constexpr size_t SCRATCH_BYTES = 64 * (SCRATCH_RANKS + 1) + 64;
    void* scratch = nullptr;
    int enable_p2p(size_t rec_bytes, hipStream_t st, double timeout_s);
    // single-process multi-device (elp_control.ngpu): the group allocated this
    // rank's mailbox and the device array of every rank's mailbox (raw peer
    // pointers after hipDeviceEnablePeerAccess, no IPC) and proved the round
    // trip; the communicator takes ownership of both
    void adopt_p2p(void* mine, void** dpeers_dev);
    double rtt_us = 0.0;  // the probe's measured exchange round (k_mbox_probe), 0 when none
    // ngpu on distinct devices: a rank failed while its peers wait inside an
    // RCCL collective -- ncclCommAbort releases them; the communicator is then
    // unusable (every later collective fails).  Called from another rank's
    // thread: `aborted` is atomic and every collective tests it before it
    // touches `nccl`, which abort_rccl never clears (the handle stays valid to
    // read; RCCL fails the calls on an aborted communicator)
    void abort_rccl();
    std::atomic<bool> aborted{false};

    static int unique_id(uint8_t id[128]);
    int init_rccl(const uint8_t id[128], int world_size, int rank_);
    // a communicator of ncclCommInitAll (single-process multi-device): taken over
    int adopt_rccl(void* comm, int world_size, int rank_);
    // ncclCommInitAll over devs (one communicator per device, rank = position)
    static int init_all(std::vector<void*>& comms, const std::vector<int>& devs);
    int init_host(int world_size, int rank_, elp_host_allgather_fn ag, elp_host_allreduce_fn ar,
                  elp_host_bcast_fn bc, void* user);
    void destroy();
    // recv holds world * bytes; send is this rank's record
    int allgather(const void* dsend, void* drecv, size_t bytes, hipStream_t st);
    int allreduce_sum_f64(double* dbuf, size_t count, hipStream_t st);
    int allreduce_max_i32(int32_t* dbuf, size_t count, hipStream_t st);
    int bcast_f64(double* dbuf, size_t count, int root, hipStream_t st);
};

// Mailbox round-trip probe (k_mbox_probe): thread t stores the reserved
// sequence word into this rank's slots of peers[t]'s mailbox and waits (ticks
// of the 100 MHz clock at most) for rank t's word in `mine`; ok[0] = 1 when all
// arrived, ok[1] = 100 MHz ticks of MBOX_ROUNDS timed exchange rounds after it
// (mbox_rtt_us: microseconds per round).  Every rank's probe must be in flight
// at the same time; ok holds 2 ints.
hipError_t launch_mbox_probe(void* const* dpeers, void* mine, int P, int rank, int64_t rec_bytes, int32_t* ok,
                             unsigned long long ticks, hipStream_t st);
double mbox_rtt_us(int32_t ticks);

}  // namespace elp
