// elp_comm.hip -- communicator stub for world size 1 (multi-GPU: see DESIGN.md).
#include "elp_comm.h"

#include <cstring>

#include "../../include/easylp_hip.h"

namespace elp {

int Comm::unique_id(uint8_t id[128]) {
    std::memset(id, 0, 128);
    return ELP_E_UNSUPPORTED;
}
int Comm::init(const uint8_t*, int world_size, int rank_) {
    if (world_size == 1) {
        world = 1;
        rank = rank_;
        return 0;
    }
    return ELP_E_UNSUPPORTED;
}
void Comm::destroy() {}
int Comm::allreduce_max_int(int v, hipStream_t) { return v; }
int Comm::allgather_shards(double*, int64_t, hipStream_t) { return 0; }

}  // namespace elp
