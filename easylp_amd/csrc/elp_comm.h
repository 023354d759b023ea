// elp_comm.h -- column-shard communicator.
// World size 1 is a no-op; the RCCL path is added in elp_comm.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace elp {

struct Comm {
    int world = 1, rank = 0;
    void* nccl = nullptr;  // ncclComm_t
    static int unique_id(uint8_t id[128]);
    int init(const uint8_t id[128], int world_size, int rank_);
    void destroy();
    int allreduce_max_int(int v, hipStream_t st);
    int allgather_shards(double* x, int64_t n, hipStream_t st);
};

}  // namespace elp
