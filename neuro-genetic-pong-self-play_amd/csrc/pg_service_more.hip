// pg_service_more.hip -- k_service (pg_service.hpp) for every split layout
// but the bench one: L = 8 lanes per game with U = 1..8 units per lane
// (H <= 32) or U = 16 with 2 or 4 outputs, and L = 16, 32, 64 (H <= 256).  Built with the default
// scheduler (see pg_service.hpp); pong_ga.hip's launch_service_any calls in
// here for these layouts.
#include "pg_service.hpp"

namespace pg {

template <typename WT>
static int32_t launch_more(const EvalParams &p, int L, int O, hipStream_t s) {
  const int H = p.nodes[1];
#define PG_SVC(LL, UU)                                                   \
  if (L == LL && (LL / 2) * UU >= H) {                                   \
    if (O == 2) return launch_service<LL, UU, 2, WT>(p, s);              \
    if (O == 3) return launch_service<LL, UU, 3, WT>(p, s);              \
    if (O == 4) return launch_service<LL, UU, 4, WT>(p, s);              \
  }
  if (L == 8 && H > 32 && H <= 64) {  // the bench layout's O = 2 / 4 instances (O = 3: pong_ga.hip)
    if (O == 2) return launch_service<8, 16, 2, WT>(p, s);
    if (O == 4) return launch_service<8, 16, 4, WT>(p, s);
  }
  PG_SVC(8, 1) PG_SVC(8, 2) PG_SVC(8, 4) PG_SVC(8, 8) PG_SVC(16, 1) PG_SVC(16, 2) PG_SVC(16, 4) PG_SVC(16, 8)
  PG_SVC(32, 1) PG_SVC(32, 2) PG_SVC(32, 4) PG_SVC(32, 8) PG_SVC(64, 1) PG_SVC(64, 2) PG_SVC(64, 4) PG_SVC(64, 8)
#undef PG_SVC
  return fail(PG_ERR_UNSUPPORTED, "no service kernel for L=%d H=%d O=%d", L, H, O);
}

int32_t launch_service_more(const EvalParams &p, int L, int O, bool f64, hipStream_t s) {
  return f64 ? launch_more<double>(p, L, O, s) : launch_more<float>(p, L, O, s);
}

}  // namespace pg
