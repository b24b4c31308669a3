// bm_guided.hip — placeholder until the fused guided kernel lands.
#include "bm_guided.h"

namespace sm {

void guided_workspace_free(GuidedWorkspace& ws) {
    if (ws.stats) (void)hipFree(ws.stats);
    ws.stats = nullptr;
    ws.stats_bytes = 0;
}

hipError_t launch_guided_match(GuidedWorkspace&, const uint8_t*, const uint8_t*, int, int, int, int, int64_t, int,
                               int, float, int, uint8_t*, int, int64_t, hipStream_t) {
    return hipErrorNotSupported;
}

}  // namespace sm
