// pg_device.hpp -- device-side building blocks of the GA evaluation loop for
// gfx950 (MI355X): the struct-of-arrays Pong stepper, the observation
// features, the scripted opponents and wave-level reductions.
//
// Reference behaviour each piece reproduces is cited inline (file:line in
// n00b001/neuro-genetic-pong-self-play).  The physics is the build's own
// (DESIGN.md "Physics"): the reference steps the absent gym-retro emulator.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pg_f64math.h"

namespace pg {

// A test every lane of the wave evaluates, taken as a wave-uniform branch: a
// wave where no lane needs the guarded block skips it with one scalar branch
// instead of the exec-mask save / restore of a divergent one.  Use as
// `if (PG_ANY(c) && c) { ... }` for blocks most frames skip.
#define PG_ANY(c) __builtin_expect(__builtin_amdgcn_ballot_w64(c) != 0, 0)

// ---- playfield geometry: the 160x160 crop (rows 34..193) of obs.npy ----
constexpr int kFieldW = 160;
constexpr int kFieldH = 160;
constexpr int kPaddleH = 16;
constexpr int kPaddleW = 4;
constexpr int kLeftPaddleX = 16;    // columns 16..19
constexpr int kRightPaddleX = 140;  // columns 140..143
constexpr int kBallH = 4;
constexpr int kBallW = 2;
constexpr int kPaddleYMin = -8;
constexpr int kPaddleYMax = 152;
constexpr int kPaddleSpeed = 3;
constexpr int kCpuSpeed = 2;
constexpr int kServeDelay = 30;
constexpr int kBallVx0 = 2;
constexpr int kBallVxMax = 4;
constexpr int kDoneScore = 21;
// ---- episode constants (config.py) ----
constexpr int kWinScore = 3;          // WIN_SCORE config.py:53
constexpr int kTimeoutThresh = 2000;  // TIMEOUT_THRESH config.py:28

enum : int { kOppHard = 0, kOppRomCpu = 1, kOppScore = 2, kOppNN = 3 };
// Pong::step's result; kStepRally: a bounce at or past the point's
// kRallyHits-th return (PongK::step only: k_service's rally check)
enum : int { kStepFly = 0, kStepBounce = 1, kStepPoint = 2, kStepRally = 3 };
// k_service's serve table: game slots and points per slot (a game serves at
// most 41 times: done() at 21 points)
constexpr int kServeTabSlots = 16, kServeTabPoints = 64;

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Physics seed of game slot g (main.py:33): independent of the genome, as the
// emulator started from a state file is deterministic.
__host__ __device__ inline uint64_t game_seed(uint64_t base, int g) {
  return splitmix64(base ^ (0xA24BAED4963EE407ull * (uint64_t)(g + 1)));
}

__device__ inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// One game's state: 16 x 32-bit words, the SoA row of pg_physics_* (64 B).
struct Pong {
  int bx, by, vx, vy, vis, timer, dir, hits, point, lpy, rpy, s1, s2, one_player;
  uint64_t seed;

  __device__ void reset(uint64_t s, int one_p) {
    bx = 79; by = 78; vx = 0; vy = 0; vis = 0; timer = kServeDelay; dir = 1; hits = 0; point = 0;
    lpy = 72; rpy = 72; s1 = 0; s2 = 0; one_player = one_p; seed = s;
  }

  __device__ bool done() const { return s1 >= kDoneScore || s2 >= kDoneScore; }

  __device__ static int dy_of(int code) {  // code: 0 = [0,0], 1 = [1,0] up, 2 = [0,1] down, 3 = [1,1]
    return (code == 2) - (code == 1);
  }
  // the row clamp of a paddle top: one v_med3_i32 (the upper bound from an
  // SGPR: a gfx9 VOP3 takes no literal, so min(max()) compiled to two ops)
  __device__ static int clamp_row(int y) {
#if defined(__HIP_DEVICE_COMPILE__)
    int r;
    asm("v_med3_i32 %0, %1, -8, %2" : "=v"(r) : "v"(y), "s"(kPaddleYMax));
    static_assert(kPaddleYMin == -8, "the inline constant above");
    return r;
#else
    return min(max(y, kPaddleYMin), kPaddleYMax);
#endif
  }
  __device__ static int move(int y, int dy, int speed) { return clamp_row(y + dy * speed); }
  // a player's move for action code c: 0, -3, +3, 0 rows (dy_of(c) * kPaddleSpeed
  // as one signed bitfield extract from a byte table)
  __device__ static int move_player(int y, int code) {
    static_assert(kPaddleSpeed == 3, "the table below");
    return clamp_row(y + __builtin_amdgcn_sbfe(0x0003FD00, 8 * code, 8));
  }

  // env.step(action) (main.py:77): right [up,down] = action[4:6], left = action[6:8].
  // The common case -- the ball in flight, away from both paddle faces -- is
  // straight-line code; reaching a face (bounce or miss, ~1 frame in 40 of a
  // game) and the hidden-ball countdown are wave-uniform branches (PG_ANY):
  // they cost only the waves where some game takes them.  Returns what the
  // frame did at a face: kStepBounce (a paddle returned the ball), kStepPoint
  // (a miss: exactly one score grew), else kStepFly -- so a caller needs no
  // copies of hits and the scores from before the step.
  __device__ int step(int right_code, int left_code) {
    return step(right_code, left_code, [this](int pt) { return serve_entry(seed, pt); });
  }
  // the same with the serves read from a table: serve_of(point) = serve_entry(seed, point)
  template <class ServeOf>
  __device__ int step(int right_code, int left_code, ServeOf serve_of) {
    return step(right_code, left_code, serve_of, PG_ANY(one_player != 0));
  }
  // any_one_player: wave-uniform, true when some game of the wave may be a
  // 1-player env (k_service keeps it from its game starts: no test per frame)
  template <class ServeOf>
  __device__ int step(int right_code, int left_code, ServeOf serve_of, bool any_one_player) {
    int ev = kStepFly;
    rpy = move_player(rpy, right_code);
    // left paddle: the action, or the built-in CPU of the 1-player env
    // (main.py:40) -- behind a wave-uniform test: no game of a self-play
    // schedule takes it
    int nl = move_player(lpy, left_code);
    if (__builtin_expect(any_one_player, 0)) {
      const int bc2 = 2 * by + kBallH - 1, pc2 = 2 * lpy + kPaddleH - 1;
      const int cpu_dy = vis ? ((bc2 < pc2 - 4) ? -1 : ((bc2 > pc2 + 4) ? 1 : 0)) : 0;
      nl = one_player ? move(lpy, cpu_dy, kCpuSpeed) : nl;
    }
    lpy = nl;

    constexpr int ymax = kFieldH - kBallH;
    constexpr int lface = kLeftPaddleX + kPaddleW, rface = kRightPaddleX;
    // ball in play: move, walls; the plain flight as selects, reaching a face
    // and the hidden ball behind wave-uniform tests (no exec-mask juggling on
    // the frames where no game of the wave needs them)
    const bool play = vis != 0;
    const int nx = bx + vx;
    int ny = by + vy;
    const bool wall_top = ny < 0, wall_bot = ny > ymax;
    ny = wall_top ? -ny : (wall_bot ? 2 * ymax - ny : ny);
    const int wvy = (wall_top || wall_bot) ? -vy : vy;
    const bool to_left = play && (vx < 0) && (nx <= lface - 1);
    const bool to_right = play && (vx > 0) && (nx + kBallW - 1 >= rface);
    const bool face = to_left || to_right;
    const bool fly = play && !face;
    bx = fly ? nx : bx;
    by = fly ? ny : by;
    vy = fly ? wvy : vy;
    // the rare blocks -- a paddle face reached, the ball hidden -- behind one
    // wave-uniform test (play is the state before this frame: the frame of a
    // miss only starts the serve timer)
    if (PG_ANY(face || !play)) {
    if (face) {  // crossing a paddle face: bounce or miss
      const int py = to_left ? lpy : rpy;
      if ((ny <= py + kPaddleH - 1) && (ny + kBallH - 1 >= py)) {  // rows overlap: bounce
        hits += 1;
        const int mag = min(kBallVx0 + (hits >> 2), kBallVxMax);
        // (2 (ny - py) - 12) / 6 truncated toward zero; |d| <= 18 is even, so |d| / 6 == (|d| * 43) >> 8
        const int d = 2 * (ny - py) - 12;
        const int q = (abs(d) * 43) >> 8;
        bx = to_left ? lface : rface - kBallW;
        by = ny;
        vx = to_left ? mag : -mag;
        vy = d < 0 ? -q : q;
        ev = kStepBounce;
      } else {  // a miss scores for the other side; the ball stays, hidden until the next serve
        s2 += to_left ? 1 : 0;
        s1 += to_right ? 1 : 0;
        dir = to_left ? -1 : 1;
        timer = kServeDelay;
        vis = 0;
        ev = kStepPoint;
      }
    }
    if (!play) {
      // ball hidden: the serve timer runs down (the frame of a miss only starts it)
      timer = timer > 0 ? timer - 1 : 0;
      if (timer == 0 && !done()) serve_from(serve_of(point));
    }
    }
    return ev;
  }

  // Top row of a paddle after h frames of clamp-only actions: with the ball
  // hidden get_actions returns [0,0] (main.py:151-153) and
  // keep_within_game_bounds_please (utils.py:71-77) moves a paddle whose
  // centroid is < 16 down and > 144 up -- rows <= 8 down, rows >= 137 up, 3 px
  // a frame (move() never clamps there) -- until it is inside [9, 136].
  __device__ static int drift(int py, int h) {
    const int down = py <= 8 ? min((11 - py) / 3, h) : 0;   // ceil((9 - py) / 3) frames
    const int up = py >= 137 ? min((py - 134) / 3, h) : 0;  // ceil((py - 136) / 3) frames
    return py + kPaddleSpeed * (down - up);
  }

  // The (point + 1)-th serve of a game with physics seed s: the ball's row in
  // bits 0-7, vy + 2 in bits 8-15.  A function of (seed, point) only, so
  // k_service tabulates it per game slot once per launch (pg_service.hpp).
  __host__ __device__ static uint32_t serve_entry(uint64_t s, int pt) {
    const uint64_t r = splitmix64(s ^ ((uint64_t)(pt + 1) * 0xD1B54A32D192ED03ull));
    const int sel = (int)((r >> 32) & 3u);
    const int row = 40 + (int)(r % 77u);
    const int v = sel < 2 ? sel - 2 : sel - 1;  // {-2, -1, 1, 2}
    return (uint32_t)row | ((uint32_t)(v + 2) << 8);
  }
  __device__ void serve_from(uint32_t e) {
    bx = 79;
    by = (int)(e & 255u);
    vy = (int)(e >> 8) - 2;
    vx = dir * kBallVx0;
    hits = 0;
    vis = 1;
    point += 1;
  }
  __device__ void serve() { serve_from(serve_entry(seed, point)); }
};

// ---- periodic rallies (DESIGN.md "Periodic rallies") ----
// Everything that decides the rest of an episode while no point is scored:
// the Pong state after a frame's step and the two actions decided in that
// frame (the next frame's "last ball" is this state's ball).  hits only acts
// through min(2 + hits/4, 4), so it is capped at 8; the scores, seed and
// player mode are constant between points.  61 bits; injective on reachable
// states (bx < 160, by < 157, |vx| <= 4, |vy| <= 3, timer <= 30, point <= 42,
// paddle top in [-8, 152]).  Two equal keys at two frames of one point mean
// the rally is periodic: no point is ever scored again, and the game ends at
// the frame where the no-score counter passes TIMEOUT_THRESH (main.py:102-107).
__device__ inline uint64_t rally_key(const Pong &s, int act_r, int act_l) {
  uint64_t k = (uint64_t)(s.bx & 255);
  k = (k << 8) | (uint64_t)(s.by & 255);
  k = (k << 4) | (uint64_t)(s.vx & 15);
  k = (k << 4) | (uint64_t)(s.vy & 15);
  k = (k << 1) | (uint64_t)(s.vis & 1);
  k = (k << 5) | (uint64_t)(s.timer & 31);
  k = (k << 1) | (uint64_t)(s.dir > 0);
  k = (k << 4) | (uint64_t)(s.hits < 8 ? s.hits : 8);
  k = (k << 6) | (uint64_t)(s.point & 63);
  k = (k << 8) | (uint64_t)((s.lpy + 8) & 255);
  k = (k << 8) | (uint64_t)((s.rpy + 8) & 255);
  k = (k << 2) | (uint64_t)(act_r & 3);
  k = (k << 2) | (uint64_t)(act_l & 3);
  return k;
}
// Brent's cycle search over one point: the key is saved when the no-score
// counter reaches kRallyStart (k_wide) or at the point's kRallyHits-th return
// (k_service) and re-saved each time the distance doubles.  k_wide compares
// keys every kRallyStride frames (a multiple of the period is then still met
// within kRallyStride periods); k_service at the frames where a paddle
// returns the ball (pg_service.hpp).
#ifndef PG_RALLY_START
#define PG_RALLY_START 256
#endif
#ifndef PG_RALLY_STRIDE
#define PG_RALLY_STRIDE 4
#endif
constexpr int kRallyStart = PG_RALLY_START;
constexpr int kRallyStride = PG_RALLY_STRIDE;
// k_service: the search opens at a point's kRallyHits-th return (the first
// bounce whose state can recur: rally_key caps hits there) with a first span
// of kRallySpan0 frames
#ifndef PG_RALLY_SPAN0
#define PG_RALLY_SPAN0 64
#endif
constexpr int kRallyHits = 8;
static_assert(kRallyHits <= 8, "rally_key caps hits at 8");
constexpr int kRallySpan0 = PG_RALLY_SPAN0;

// Doubled centroid row of a paddle clipped to rows [0,160): what
// get_rect_quickly (utils.py:60-68) returns for the rendered rectangle, x2.
__device__ inline int paddle_c2(int py) {
  const int lo = py < 0 ? 0 : py;
  const int hi = py + kPaddleH - 1 > kFieldH - 1 ? kFieldH - 1 : py + kPaddleH - 1;
  return lo + hi;
}

// keep_within_game_bounds_please (utils.py:71-77): centroid < 16 -> down,
// > 144 -> up.  In doubled units: c2 < 32, c2 > 288.
__device__ inline int clamp_action(int c2, int code) {
  return c2 < 32 ? 2 : (c2 > 2 * (kFieldH - 16) ? 1 : code);
}
// The same on k_service's actions, kept as the paddle's move in centroid
// units (doubled rows): up -6, down +6, no-op 0 -- the step adds it as is.
__device__ inline int clamp_move(int c2, int move) {
  static_assert(kPaddleSpeed == 3, "doubled moves of 6");
  return c2 < 32 ? 6 : (c2 > 2 * (kFieldH - 16) ? -6 : move);
}
// the action code (1 up, 2 down, 0 none) of a move: the trace and rally_key
__device__ inline int move_code(int move) { return move < 0 ? 1 : (move > 0 ? 2 : 0); }

// HardcodedAi.run (dumb_ais.py:2-8) on inference() features: compares
// ball_y/160 (x[1]) with me/160 (x[4]); the /160 is monotone, so the doubled
// integer centroids compare the same way.
__device__ inline int hardcoded(int by2, int me2) { return by2 < me2 ? 1 : (by2 > me2 ? 2 : 0); }
__device__ inline int hardcoded_move(int by2, int me2) { return by2 < me2 ? -6 : (by2 > me2 ? 6 : 0); }

// argmax index -> action code (numpy_nn.py:131-137; index >= 2 -> no-op, the
// build's extension for 3-output networks).
__device__ inline int index_to_code(int idx) {  // 0 -> 1, 1 -> 2, 2, 3 -> 0: bits 2 idx of 0b1001
  return (int)__builtin_amdgcn_ubfe(9u, 2u * (unsigned)idx, 2u);
}
__device__ inline int index_to_move(int idx) {  // clamp_move's units: signed byte idx of 0x0006FA
  return (int)__builtin_amdgcn_sbfe(0x0006FA, 8u * (unsigned)idx, 8u);
}

// ---- k_service's game state: Pong in the doubled units of the features ----
// The same game as Pong, kept as the values the networks read: the ball's
// doubled centroid (bx2 = 2 bx + kBallW - 1, by2 = 2 by + kBallH - 1), its
// doubled velocity, and each paddle's doubled centroid 2 py + kPaddleH - 1 --
// so a frame's features (utils.py:139-153) need no arithmetic.  Conventions
// of k_service that the general step does not assume:
//  * actions as the paddle's move in centroid units (clamp_move: -6, 0, +6);
//  * the action-driven paddles stay inside the clamp band:
//    keep_within_game_bounds_please (utils.py:71-77, clamp_move) forces a
//    paddle whose top row is <= 8 (c2 <= 31) down and one whose top row is
//    >= 137 (c2 >= 289) up, 3 rows a frame, every frame; from the reset row 72
//    a paddle's top row stays in [6, 139] (from [9, 136] a move reaches
//    [6, 139], from [6, 8] / [137, 139] the forced move returns it to
//    [9, 136]; the serve-delay drift ends inside [9, 136]), where the
//    rectangle is never clipped (c2 is the feature) and the row clamp
//    [-8, 152] never acts.  The built-in CPU paddle of a 1-player env leaves
//    the band: its c2 is the unclipped 2 py + 15 and c2_clip gives the feature;
//  * a ball in play lies between the faces (bx in [lface, rface - kBallW]:
//    served at 79, moved only while it stays there, put on a face at a
//    bounce), so with |vx| <= kBallVxMax it can only cross the face it moves
//    towards -- one range test, no sign tests; and the moved position is
//    stored whatever the frame does: a bounce overwrites it, a hidden ball's
//    position is never read (no features; the serve sets bx, by, vx and vy);
//  * a bounce at or past the point's kRallyHits-th return reports kStepRally.
struct PongK {
  int bx2, by2, vx2, vy2, vis, timer, dir, hits, point, lc2, rc2, s1, s2, one_player;
  uint64_t seed;
  static_assert(kBallH == 4 && kPaddleH == 16 && kBallW == 2, "the doubled-unit constants below");
  static constexpr int kC2Reset = 2 * 72 + kPaddleH - 1;

  __device__ void reset(uint64_t s, int one_p) {
    bx2 = 2 * 79 + kBallW - 1; by2 = 2 * 78 + kBallH - 1; vx2 = 0; vy2 = 0; vis = 0; timer = kServeDelay;
    dir = 1; hits = 0; point = 0; lc2 = kC2Reset; rc2 = kC2Reset; s1 = 0; s2 = 0; one_player = one_p; seed = s;
  }
  __device__ bool done() const { return s1 >= kDoneScore || s2 >= kDoneScore; }

  // the feature of a paddle centroid kept unclipped (the 1-player CPU paddle)
  __device__ static int c2_clip(int c2) { return paddle_c2((c2 - (kPaddleH - 1)) >> 1); }
  // Pong::drift in centroid units: top row <= 8 <=> c2 <= 31, >= 137 <=> c2 >= 289;
  // (11 - py) / 3 = (37 - c2) / 6 and (py - 134) / 3 = (c2 - 283) / 6 (c2 odd)
  __device__ static int drift2(int c2, int h) {
    const int down = c2 <= 31 ? min((37 - c2) / 6, h) : 0;
    const int up = c2 >= 289 ? min((c2 - 283) / 6, h) : 0;
    return c2 + 2 * kPaddleSpeed * (down - up);
  }

  // env.step (Pong::step) on the paddles' moves; serve_of(point) = Pong::serve_entry(seed, point)
  template <class ServeOf>
  __device__ int step(int right_move, int left_move, ServeOf serve_of, bool any_one_player) {
    int ev = kStepFly;
    rc2 += right_move;
    int nl = lc2 + left_move;
    if (__builtin_expect(any_one_player, 0)) {  // the 1-player env's CPU (main.py:40), Pong::step's rule
      const int cpu_dy = vis ? ((by2 < lc2 - 4) ? -1 : ((by2 > lc2 + 4) ? 1 : 0)) : 0;
      const int moved = lc2 + 2 * kCpuSpeed * cpu_dy;
      constexpr int lo = 2 * kPaddleYMin + kPaddleH - 1, hi = 2 * kPaddleYMax + kPaddleH - 1;
      nl = one_player ? (moved < lo ? lo : (moved > hi ? hi : moved)) : nl;
    }
    lc2 = nl;

    constexpr int top2 = kBallH - 1;                              // ny < 0    <=> ny2 < top2
    constexpr int bot2 = 2 * (kFieldH - kBallH) + kBallH - 1;     // ny > ymax <=> ny2 > bot2
    constexpr int lface = kLeftPaddleX + kPaddleW, rface = kRightPaddleX;
    constexpr int left2 = 2 * (lface - 1) + kBallW - 1;           // nx <= lface - 1
    constexpr int right2 = 2 * (rface - kBallW + 1) + kBallW - 1; // nx + kBallW - 1 >= rface
    const bool play = vis != 0;
    const int nx2 = bx2 + vx2;
    int ny2 = by2 + vy2;
    const bool wall_top = ny2 < top2, wall_bot = ny2 > bot2;
    ny2 = wall_top ? 2 * top2 - ny2 : (wall_bot ? 2 * bot2 - ny2 : ny2);  // -ny, 2 ymax - ny
    vy2 = (wall_top || wall_bot) ? -vy2 : vy2;
    const bool to_left = play && nx2 <= left2;
    const bool to_right = play && nx2 >= right2;
    bx2 = nx2;
    by2 = ny2;
    if (PG_ANY(to_left || to_right || !play)) {
    if (to_left || to_right) {  // crossing a paddle face: bounce or miss
      // d = 2 (ny - py) - 12; the rows overlap iff -3 <= ny - py <= 15
      const int d = ny2 - (to_left ? lc2 : rc2);
      if (d >= -18 && d <= 18) {  // bounce
        hits += 1;
        const int mag = min(kBallVx0 + (hits >> 2), kBallVxMax);
        const int q = (abs(d) * 43) >> 8;  // |d| / 6 for even |d| <= 18
        bx2 = to_left ? 2 * lface + kBallW - 1 : 2 * (rface - kBallW) + kBallW - 1;
        vx2 = to_left ? 2 * mag : -2 * mag;
        vy2 = d < 0 ? -2 * q : 2 * q;
        ev = hits >= kRallyHits ? kStepRally : kStepBounce;
      } else {  // a miss scores for the other side; the ball is hidden until the next serve
        s2 += to_left ? 1 : 0;
        s1 += to_right ? 1 : 0;
        dir = to_left ? -1 : 1;
        timer = kServeDelay;
        vis = 0;
        ev = kStepPoint;
      }
    }
    if (!play) {
      timer = timer > 0 ? timer - 1 : 0;
      if (timer == 0 && !done()) {
        const uint32_t e = serve_of(point);
        bx2 = 2 * 79 + kBallW - 1;
        by2 = 2 * (int)(e & 255u) + kBallH - 1;
        vy2 = 2 * ((int)(e >> 8) - 2);
        vx2 = 2 * dir * kBallVx0;
        hits = 0;
        vis = 1;
        point += 1;
      }
    }
    }
    return ev;
  }

  // rally_key of the same state (Pong units)
  __device__ uint64_t key(int act_r, int act_l) const {
    Pong s;
    s.bx = (bx2 - (kBallW - 1)) >> 1;
    s.by = (by2 - (kBallH - 1)) >> 1;
    s.vx = vx2 >> 1;
    s.vy = vy2 >> 1;
    s.vis = vis;
    s.timer = timer;
    s.dir = dir;
    s.hits = hits;
    s.point = point;
    s.lpy = (lc2 - (kPaddleH - 1)) >> 1;
    s.rpy = (rc2 - (kPaddleH - 1)) >> 1;
    return rally_key(s, act_r, act_l);
  }
};

// ---- wave-level helpers ----
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over the L lanes of an aligned lane group; every lane of the group gets
// the bitwise-identical total (each butterfly/mirror step adds the same two
// operands in both partner lanes, and IEEE addition commutes).
template <int L>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (L >= 2) v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
  if constexpr (L >= 4) v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
  if constexpr (L >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror: quad <-> quad
  if constexpr (L >= 16) v += dpp_mov<0x140>(v); // row_mirror: half-row <-> half-row
  if constexpr (L >= 32) {  // rows 0<->1, 2<->3: v_permlane16_swap (gfx950)
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  if constexpr (L >= 64) {  // half-waves 0-31 <-> 32-63: v_permlane32_swap (gfx950)
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  return v;
}

template <int L>
__device__ __forceinline__ float group_max(float v) {
  if constexpr (L >= 2) v = fmaxf(v, dpp_mov<0xB1>(v));
  if constexpr (L >= 4) v = fmaxf(v, dpp_mov<0x4E>(v));
  if constexpr (L >= 8) v = fmaxf(v, dpp_mov<0x141>(v));
  if constexpr (L >= 16) v = fmaxf(v, dpp_mov<0x140>(v));
  if constexpr (L >= 32) v = fmaxf(v, __shfl_xor(v, 16, 64));
  if constexpr (L >= 64) v = fmaxf(v, __shfl_xor(v, 32, 64));
  return v;
}

// Make a group-uniform value provably wave-uniform when the group is the whole
// wave (lets hipcc keep the game state in SGPRs and branch on the scalar unit).
template <int L>
__device__ __forceinline__ int uniformize(int v) {
  if constexpr (L == 64) return __builtin_amdgcn_readfirstlane(v);
  return v;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// numpy's sigmoid 1 / (1 + np.e ** -x) (numpy_nn.py:22-23) in f64; np.e is the
// double nearest e; pow(e_d, -x) correctly rounded (pg_f64math.h).
__device__ __forceinline__ double sigmoid_f64(double z) { return pg_sigmoid_f64(z); }

// ------------------------------------------------ numpy's np.dot order ----
// Row j of np.dot(W, x) for a C-contiguous [n, m] float64 W (numpy_nn.py:127):
// numpy calls cblas_dgemv, OpenBLAS runs dgemv_t, whose x86-64 AVX2/FMA kernel
// (dgemv_t_4.c) takes the outputs 4 at a time, then 2, then 1 -- each with its
// own summation -- over blocks of <= 2048 elements, then the m & 3 tail.  The
// oracle restates the same order (or_blas_dot, pinned to np.dot by
// tests/test_blas_order.py); kinds:
//   0  j < 4 (n / 4):         s[i % 4] = fma(a_i, x_i, s[i % 4]); (s0 + s2) + (s1 + s3)
//   1  the next 2 if n & 2:   s[i % 2] += a_i x_i (product rounded);  s0 + s1
//   2  the last if n & 1:     s[i % 4] += a_i x_i;                    (s0 + s2) + (s1 + s3)
__host__ __device__ constexpr int blas_kind(int j, int n) {
  return j < 4 * (n >> 2) ? 0 : (((n & 2) && j < 4 * (n >> 2) + 2) ? 1 : 2);
}

// One block's partial sums (nb a multiple of 4) starting at element i0.
template <class AF, class XF>
__device__ __forceinline__ double blas_block(AF a, XF x, int i0, int nb, int kind) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (kind == 0) {
#pragma unroll 2
    for (int i = i0; i < i0 + nb; i += 4) {
      s0 = fma(a(i), x(i), s0);
      s1 = fma(a(i + 1), x(i + 1), s1);
      s2 = fma(a(i + 2), x(i + 2), s2);
      s3 = fma(a(i + 3), x(i + 3), s3);
    }
    return __dadd_rn(__dadd_rn(s0, s2), __dadd_rn(s1, s3));
  }
  if (kind == 1) {
#pragma unroll 2
    for (int i = i0; i < i0 + nb; i += 2) {
      s0 = __dadd_rn(s0, __dmul_rn(a(i), x(i)));
      s1 = __dadd_rn(s1, __dmul_rn(a(i + 1), x(i + 1)));
    }
    return __dadd_rn(s0, s1);
  }
#pragma unroll 2
  for (int i = i0; i < i0 + nb; i += 4) {
    s0 = __dadd_rn(s0, __dmul_rn(a(i), x(i)));
    s1 = __dadd_rn(s1, __dmul_rn(a(i + 1), x(i + 1)));
    s2 = __dadd_rn(s2, __dmul_rn(a(i + 2), x(i + 2)));
    s3 = __dadd_rn(s3, __dmul_rn(a(i + 3), x(i + 3)));
  }
  return __dadd_rn(__dadd_rn(s0, s2), __dadd_rn(s1, s3));
}

// The m & 3 trailing elements at i0 added to y (dgemv_t_4.c's tail, as GCC
// contracts it): 1: fma(a, x, y); 2: y + fma(a0, x0, a1 x1);
// 3: y + fma(a2, x2, fma(a0, x0, a1 x1)).
template <class AF, class XF>
__device__ __forceinline__ double blas_tail(AF a, XF x, int i0, int m3, double y) {
  if (m3 == 1) return fma(a(i0), x(i0), y);
  if (m3 == 0) return y;
  const double t = fma(a(i0), x(i0), __dmul_rn(a(i0 + 1), x(i0 + 1)));
  return __dadd_rn(y, m3 == 2 ? t : fma(a(i0 + 2), x(i0 + 2), t));
}

// A hidden unit of the game networks: np.dot over [x0..x5] (+ the bias weight
// times 1.0 when b).  m = 6 or 7: one 4-element block -- the same
// (p0 + p2) + (p1 + p3) for every kind -- then the 2- or 3-element tail.
__device__ __forceinline__ double blas_dot6(const double w[7], const double x[6], int b) {
  const double blk = __dadd_rn(__dadd_rn(__dmul_rn(w[0], x[0]), __dmul_rn(w[2], x[2])),
                               __dadd_rn(__dmul_rn(w[1], x[1]), __dmul_rn(w[3], x[3])));
  const double t = fma(w[4], x[4], __dmul_rn(w[5], x[5]));
  return __dadd_rn(blk, b ? fma(w[6], 1.0, t) : t);
}

// y_j = np.dot(W, x)[j], a(i) = W[j][i], x(i) = x[i], i < m.
template <class AF, class XF>
__device__ __forceinline__ double blas_dot(AF a, XF x, int m, int kind) {
  const int m3 = m & 3, m2 = (m & 2047) - m3;
  int m1 = m & ~3, nb = 2048, i0 = 0;
  double y = 0.0;
  while (nb == 2048) {
    m1 -= nb;
    if (m1 < 0) {
      if (m2 == 0) break;
      nb = m2;
    }
    y = __dadd_rn(y, blas_block(a, x, i0, nb, kind));
    i0 += nb;
  }
  return blas_tail(a, x, i0, m3, y);
}

}  // namespace pg
