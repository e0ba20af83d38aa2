// pg_service_more.hip -- k_service (pg_service.hpp) for every split layout
// but the bench one: L = 8 lanes per game with U = 1..8 units per lane
// (H <= 32) or U = 16 with 2 or 4 outputs, and L = 16, 32, 64 (H <= 256).  Built with the default
// scheduler (see pg_service.hpp); pong_ga.hip's launch_service_any calls in
// here for these layouts.
//
// One translation unit per (L, genome type): pong_amd/build.py compiles this
// file eight times with -DPG_MORE_L=8|16|32|64 -DPG_MORE_F64=0|1 (the ~100
// instantiations took 10 minutes as one unit, ~1.5 minutes split in parallel);
// the -DPG_MORE_DISPATCH unit (L = 8, f64) also holds launch_service_more.
#include <type_traits>

#include "pg_service.hpp"

#if !defined(PG_MORE_L) || !defined(PG_MORE_F64)
#error "build with -DPG_MORE_L=<8|16|32|64> -DPG_MORE_F64=<0|1> (pong_amd/build.py)"
#endif

namespace pg {

#define PG_MORE_CAT2(a, b, c) a##b##_##c
#define PG_MORE_CAT(a, b, c) PG_MORE_CAT2(a, b, c)
#define PG_MORE_FN PG_MORE_CAT(launch_more_L, PG_MORE_L, PG_MORE_F64)

int32_t PG_MORE_FN(const EvalParams &p, int O, hipStream_t s) {
  using WT = std::conditional<PG_MORE_F64 != 0, double, float>::type;
  constexpr int L = PG_MORE_L;
  const int H = p.nodes[1];
#define PG_SVC(UU)                                                       \
  if ((L / 2) * UU >= H) {                                               \
    if (O == 2) return launch_service<L, UU, 2, WT>(p, s);               \
    if (O == 3) return launch_service<L, UU, 3, WT>(p, s);               \
    if (O == 4) return launch_service<L, UU, 4, WT>(p, s);               \
  }
  if constexpr (L == 8) {
    if (H > 32 && H <= 64) {  // the bench layout's O = 2 / 4 instances (O = 3: pong_ga.hip)
      if (O == 2) return launch_service<8, 16, 2, WT>(p, s);
      if (O == 4) return launch_service<8, 16, 4, WT>(p, s);
      return fail(PG_ERR_UNSUPPORTED, "no service kernel for L=%d H=%d O=%d", L, H, O);
    }
  }
  PG_SVC(1) PG_SVC(2) PG_SVC(4) PG_SVC(8)
#undef PG_SVC
  return fail(PG_ERR_UNSUPPORTED, "no service kernel for L=%d H=%d O=%d", L, H, O);
}

#ifdef PG_MORE_DISPATCH
#define PG_MORE_DECL(LL)                                                  \
  int32_t launch_more_L##LL##_0(const EvalParams &p, int O, hipStream_t s); \
  int32_t launch_more_L##LL##_1(const EvalParams &p, int O, hipStream_t s);
PG_MORE_DECL(8) PG_MORE_DECL(16) PG_MORE_DECL(32) PG_MORE_DECL(64)
#undef PG_MORE_DECL

int32_t launch_service_more(const EvalParams &p, int L, int O, bool f64, hipStream_t s) {
  switch (L) {
    case 8: return f64 ? launch_more_L8_1(p, O, s) : launch_more_L8_0(p, O, s);
    case 16: return f64 ? launch_more_L16_1(p, O, s) : launch_more_L16_0(p, O, s);
    case 32: return f64 ? launch_more_L32_1(p, O, s) : launch_more_L32_0(p, O, s);
    case 64: return f64 ? launch_more_L64_1(p, O, s) : launch_more_L64_0(p, O, s);
  }
  return fail(PG_ERR_UNSUPPORTED, "no service kernel for L=%d H=%d O=%d", L, p.nodes[1], O);
}
#endif

}  // namespace pg
