// hbm_ceiling.hip -- the HBM read rate this box reaches with k_wide's load
// shape: every wave instruction a 1-KB line-aligned contiguous piece (16 B per
// lane, non-temporal), a persistent grid of 512-thread workgroups (k_wide's
// block size, one per CU by default), several pieces in flight per wave.  The
// buffer (default 8 GiB) is far past the 256 MiB Infinity Cache, and each
// byte is read once per pass, so the rate is HBM-served.  Reported beside
// k_wide's weight stream (BASELINE config 5) as the measured ceiling.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/hbm_ceiling tools/hbm_ceiling.hip
//   tools/bin/hbm_ceiling [GiB=8] [passes=5] [blocks_per_cu=1] [in_flight=4]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int F>
__global__ __launch_bounds__(512) void k_stream(const f4 *__restrict__ buf, long n_pieces, float *out) {
  // piece = 64 float4 = 1 KB, one wave instruction; wave w of the grid takes
  // pieces w, w + W, ... in groups of F issued together
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long waves = (long)gridDim.x * (blockDim.x >> 6);
  float acc = 0.f;
  for (long p0 = wave; p0 < n_pieces; p0 += waves * F) {
    f4 v[F];
#pragma unroll
    for (int f = 0; f < F; ++f) {
      const long p = p0 + (long)f * waves;
      v[f] = p < n_pieces ? __builtin_nontemporal_load(buf + p * 64 + lane) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int f = 0; f < F; ++f) acc += v[f].x + v[f].y + v[f].z + v[f].w;
  }
  if (acc == 1234.5f) out[0] = acc;  // keeps the loads (never true for this buffer)
}

int main(int argc, char **argv) {
  const double gib = argc > 1 ? std::atof(argv[1]) : 8.0;
  const int passes = argc > 2 ? std::atoi(argv[2]) : 5;
  const int per_cu = argc > 3 ? std::atoi(argv[3]) : 1;
  const int flight = argc > 4 ? std::atoi(argv[4]) : 4;
  const size_t bytes = (size_t)(gib * (1ull << 30)) / 1024 * 1024;
  const long n_pieces = (long)(bytes / 1024);
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  f4 *buf;
  float *out;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&out, sizeof(float)));
  CHECK(hipMemset(buf, 0x11, bytes));  // nonzero bytes (no zero-page shortcut can apply)
  const int grid = prop.multiProcessorCount * per_cu;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto launch = [&]() {
    if (flight == 1) hipLaunchKernelGGL(k_stream<1>, dim3(grid), dim3(512), 0, 0, buf, n_pieces, out);
    else if (flight == 2) hipLaunchKernelGGL(k_stream<2>, dim3(grid), dim3(512), 0, 0, buf, n_pieces, out);
    else if (flight == 8) hipLaunchKernelGGL(k_stream<8>, dim3(grid), dim3(512), 0, 0, buf, n_pieces, out);
    else hipLaunchKernelGGL(k_stream<4>, dim3(grid), dim3(512), 0, 0, buf, n_pieces, out);
  };
  launch();  // warm-up
  CHECK(hipDeviceSynchronize());
  std::vector<float> ms(passes);
  for (int i = 0; i < passes; ++i) {
    CHECK(hipEventRecord(a));
    launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    CHECK(hipEventElapsedTime(&ms[i], a, b));
  }
  float best = ms[0], sum = 0.f;
  for (float m : ms) {
    best = m < best ? m : best;
    sum += m;
  }
  std::printf("{\"bytes\": %zu, \"passes\": %d, \"grid\": %d, \"block\": 512, \"pieces_in_flight_per_wave\": %d, "
              "\"best_ms\": %.4f, \"mean_ms\": %.4f, \"best_TBps\": %.4f, \"mean_TBps\": %.4f, \"cus\": %d}\n",
              bytes, passes, grid, flight, best, sum / passes, bytes / (best * 1e-3) / 1e12,
              bytes / (sum / passes * 1e-3) / 1e12, prop.multiProcessorCount);
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
