// pg_pixels.hip -- the pixel path: render Pong frames from the SoA game state
// and find_stuff (utils.py:14-19 -> get_rect_quickly utils.py:60-68) over
// batches of 210x160x3 frames.
//
// The evaluation kernels never look at pixels: they use the analytic
// centroids of the rendered rectangles (DESIGN.md "Physics").  This path is
// the fidelity check of that shortcut against the reference's own pixel
// pipeline, and a batched find_stuff for frames from elsewhere (obs.npy).
// Both kernels are byte-streaming (HBM-bound): 100 800 B written per rendered
// frame, 76 800 B (the crop) read per find_stuff frame.
//
// get_rect_quickly matches PER CHANNEL: np.argwhere(crop == colour) yields
// one (row, col, channel) triple for every channel equal to the colour's, so
// a pixel counts once per matching channel; the centroid is
// (sum rows, sum cols) / count over those triples, None when count = 0.
// Integer sums are exact in f64, so (double)sum / count is numpy's value.
#include <hip/hip_runtime.h>

#include "pg_eval.hpp"

namespace pg {

constexpr int kFrameH = 210, kFrameW = 160, kFrameBytes = kFrameH * kFrameW * 3;  // obs.npy layout
constexpr int kCropTop = 34, kCropRows = 160;  // GAME_TOP .. GAME_BOTTOM (config.py)
constexpr int kGroupPix = 16, kGroupBytes = 48;  // 16 pixels = 3 x 16 B; a group never crosses a row
// config.py colours
__constant__ uint8_t kColours[4][3] = {{144, 72, 17},    // BG_COLOUR
                                       {236, 236, 236},  // BALL_COLOUR
                                       {213, 130, 74},   // LEFT_GUY_COLOUR
                                       {92, 186, 92}};   // RIGHT_GUY_COLOUR

// Colour index of frame pixel (row, col) for one game state (the oracle's
// render(): background, the walls outside the crop, both paddles clipped to
// the playfield, then the ball).
struct FrameState {
  int lpy, rpy, vis, by, bx;
};
__device__ __forceinline__ int pixel_colour(const FrameState &s, int row, int col) {
  int c = (row >= 24 && row < kCropTop) || row >= kCropTop + kCropRows ? 1 : 0;
  const int fr = row - kCropTop;
  if (fr >= 0 && fr < kCropRows) {
    if (col >= kLeftPaddleX && col < kLeftPaddleX + kPaddleW && fr >= max(s.lpy, 0) &&
        fr <= min(s.lpy + kPaddleH - 1, kFieldH - 1))
      c = 2;
    if (col >= kRightPaddleX && col < kRightPaddleX + kPaddleW && fr >= max(s.rpy, 0) &&
        fr <= min(s.rpy + kPaddleH - 1, kFieldH - 1))
      c = 3;
    if (s.vis && fr >= s.by && fr < s.by + kBallH && col >= s.bx && col < s.bx + kBallW) c = 1;
  }
  return c;
}

// Word j of a 16-pixel group painted in one colour (bytes 4j..4j+3 are fixed
// (pixel, channel) slots, so the pattern repeats every three words).
__device__ __forceinline__ uint32_t solid_word(int c, int j) {
  uint32_t w = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) w |= (uint32_t)kColours[c][(4 * j + b) % 3] << (8 * b);
  return w;
}

// One workgroup per frame; a thread paints a 16-pixel group (48 B, a group
// never crosses a row).  Most groups hold no object (one solid colour:
// background or wall) and come from three constant words; only groups an
// object's rectangle touches take the per-pixel path.  The wave's 64 groups
// (3 KB contiguous) are transposed through LDS so that each of its three
// 16-B stores covers 1 KB contiguously.
__global__ __launch_bounds__(256) void k_render(const int32_t *state, int n, uint8_t *frames) {
  __shared__ uint4 stage[4][192];  // per wave: 64 groups x 3 pieces
  const int f = blockIdx.x;
  if (f >= n) return;
  FrameState s;
  s.bx = state[PG_S_BALL_X * (long)n + f];
  s.by = state[PG_S_BALL_Y * (long)n + f];
  s.vis = state[PG_S_BALL_VISIBLE * (long)n + f];
  s.lpy = state[PG_S_LEFT_Y * (long)n + f];
  s.rpy = state[PG_S_RIGHT_Y * (long)n + f];
  uint4 *out = (uint4 *)(frames + (long)f * kFrameBytes);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int kGroups = kFrameH * kFrameW / kGroupPix;  // 2100
  for (int g0 = threadIdx.x - lane; g0 < kGroups; g0 += blockDim.x) {
    const int g = g0 + lane;
    const int row = g / (kFrameW / kGroupPix), col0 = (g % (kFrameW / kGroupPix)) * kGroupPix;
    const int fr = row - kCropTop;
    const bool in_crop = fr >= 0 && fr < kCropRows;
    const auto spans = [&](int x0, int w) { return x0 < col0 + kGroupPix && x0 + w > col0; };
    const bool lp = spans(kLeftPaddleX, kPaddleW) && fr >= s.lpy && fr <= s.lpy + kPaddleH - 1;
    const bool rp = spans(kRightPaddleX, kPaddleW) && fr >= s.rpy && fr <= s.rpy + kPaddleH - 1;
    const bool ball = s.vis && fr >= s.by && fr < s.by + kBallH && spans(s.bx, kBallW);
    uint32_t w[12];
    if (g < kGroups && in_crop && (lp || rp || ball)) {
#pragma unroll
      for (int q = 0; q < 12; ++q) w[q] = 0;
#pragma unroll
      for (int i = 0; i < kGroupPix; ++i) {
        const int c = pixel_colour(s, row, col0 + i);
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          const int b = 3 * i + ch;  // byte within the group, static
          w[b >> 2] |= (uint32_t)kColours[c][ch] << (8 * (b & 3));
        }
      }
    } else {  // the group's colour: pixel_colour without objects
      const bool wall = (row >= 24 && row < kCropTop) || row >= kCropTop + kCropRows;
#pragma unroll
      for (int q = 0; q < 12; ++q) w[q] = wall ? solid_word(1, q % 3) : solid_word(0, q % 3);
    }
    stage[wave][3 * lane] = make_uint4(w[0], w[1], w[2], w[3]);
    stage[wave][3 * lane + 1] = make_uint4(w[4], w[5], w[6], w[7]);
    stage[wave][3 * lane + 2] = make_uint4(w[8], w[9], w[10], w[11]);
    wave_lds_sync();
    const int pieces = 3 * (kGroups - g0 < 64 ? kGroups - g0 : 64);  // 16-B pieces of this wave's groups
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if (64 * k + lane < pieces) out[3 * g0 + 64 * k + lane] = stage[wave][64 * k + lane];
    wave_lds_sync();
  }
}

// find_stuff for one frame per workgroup: per-channel match counts and row /
// column sums of the ball, left and right colours over the crop, reduced
// exactly in integers, then mean = sum / count in f64 (NaN = None).
//
// Byte compares four at a time (SWAR): word j of a 16-pixel group holds bytes
// 4j..4j+3, i.e. fixed (pixel, channel) slots, so colour k's expected word is
// a constant E_k[j % 3].  x = w ^ E has a zero byte exactly where a channel
// matches; ((x & 0x7F..) + 0x7F..) | x has the high bit of every NONZERO byte
// set (exact, no carries between bytes).  The group's misses are counted with
// v_bcnt and their pixel indices summed with v_dot4_u32_u8 against the
// constant per-byte pixel index of word j; matches = 48 - misses, index sum =
// 360 - weighted misses.
__host__ __device__ constexpr uint32_t fs_expected(int k, int j) {  // k: 1..3 (ball, left, right)
  constexpr uint8_t c[4][3] = {{144, 72, 17}, {236, 236, 236}, {213, 130, 74}, {92, 186, 92}};
  uint32_t w = 0;
  for (int b = 0; b < 4; ++b) w |= (uint32_t)c[k][(4 * j + b) % 3] << (8 * b);
  return w;
}
__host__ __device__ constexpr uint32_t fs_pixel_index(int j) {  // pixel of each byte of word j, x 128
  uint32_t w = 0;
  for (int b = 0; b < 4; ++b) w |= (uint32_t)((4 * j + b) / 3) << (8 * b);
  return w;
}

__global__ __launch_bounds__(256) void k_find_stuff(const uint8_t *frames, int64_t stride, int n, double *out) {
  __shared__ int part[4][9];
  const int f = blockIdx.x;
  if (f >= n) return;
  const uint8_t *crop = frames + (long)f * stride + (long)kCropTop * kFrameW * 3;
  int cnt[3] = {0, 0, 0}, rs[3] = {0, 0, 0}, cs[3] = {0, 0, 0};
  constexpr int kGroups = kCropRows * kFrameW / kGroupPix;  // 1600
  for (int g = threadIdx.x; g < kGroups; g += blockDim.x) {
    const uint4 *src = (const uint4 *)(crop + (long)g * kGroupBytes);
    const uint4 a = src[0], b = src[1], c = src[2];
    const uint32_t w[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
    const int row = g / (kFrameW / kGroupPix), col0 = (g % (kFrameW / kGroupPix)) * kGroupPix;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      uint32_t miss = 0, wmiss = 0;  // missed bytes; their pixel indices x 128
#pragma unroll
      for (int j = 0; j < 12; ++j) {
        const uint32_t x = w[j] ^ fs_expected(k + 1, j % 3);
        const uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
        miss += __builtin_popcount(nz);
        wmiss = __builtin_amdgcn_udot4(nz, fs_pixel_index(j), wmiss, false);
      }
      const int m = 48 - (int)miss;
      const int mx = 360 - (int)(wmiss >> 7);
      cnt[k] += m;
      rs[k] += m * row;
      cs[k] += m * col0 + mx;
    }
  }
  int v[9] = {cnt[0], cnt[1], cnt[2], rs[0], rs[1], rs[2], cs[0], cs[1], cs[2]};
#pragma unroll
  for (int q = 0; q < 9; ++q)
    for (int off = 32; off > 0; off >>= 1) v[q] += __shfl_xor(v[q], off, 64);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < 9; ++q) part[threadIdx.x >> 6][q] = v[q];
  __syncthreads();
  if (threadIdx.x < 3) {
    const int k = threadIdx.x;
    long long tc = 0, tr = 0, tcol = 0;
    for (int w = 0; w < 4; ++w) {
      tc += part[w][k];
      tr += part[w][3 + k];
      tcol += part[w][6 + k];
    }
    const double nan = __builtin_nan("");
    out[(long)f * 6 + 2 * k] = tc ? (double)tr / (double)tc : nan;
    out[(long)f * 6 + 2 * k + 1] = tc ? (double)tcol / (double)tc : nan;
  }
}

}  // namespace pg

using namespace pg;

extern "C" {

int32_t pg_render_frames(const int32_t *state, int32_t n, uint8_t *frames, void *stream) {
  if (n < 0 || (n > 0 && (!state || !frames))) return fail(PG_ERR_INVALID, "render: state/frames NULL or n < 0");
  if (((uintptr_t)frames & 15) != 0) return fail(PG_ERR_INVALID, "render: frames must be 16-byte aligned");
  if (n == 0) return PG_OK;
  hipLaunchKernelGGL(k_render, dim3(n), dim3(256), 0, (hipStream_t)stream, state, n, frames);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_find_stuff(const uint8_t *frames, int64_t frame_stride, int32_t n, double *out, void *stream) {
  if (n < 0 || (n > 0 && (!frames || !out))) return fail(PG_ERR_INVALID, "find_stuff: frames/out NULL or n < 0");
  if (frame_stride < kFrameBytes || (frame_stride & 15) != 0 || ((uintptr_t)frames & 15) != 0)
    return fail(PG_ERR_INVALID, "find_stuff: frames need a 16-byte aligned base and stride >= %d", kFrameBytes);
  if (n == 0) return PG_OK;
  hipLaunchKernelGGL(k_find_stuff, dim3(n), dim3(256), 0, (hipStream_t)stream, frames, frame_stride, n, out);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

}  // extern "C"
