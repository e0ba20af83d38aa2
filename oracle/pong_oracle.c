/*
 * pong_oracle.c -- CPU ORACLE (test infrastructure only; see pong_oracle.h).
 *
 * Compiled with -ffp-contract=off so every f64 expression rounds exactly as
 * the reference's Python/numpy expressions do (no fused multiply-adds).
 */
#include "pong_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define OR_MAX_WIDTH 4096

uint64_t or_splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

/* Physics seed of game slot i (main.py:33 loop index).  The reference's
 * emulator is deterministic per state file, so a game depends only on its
 * slot, never on the genome's position in the population. */
uint64_t or_game_seed(uint64_t base_seed, int game_index) {
  return or_splitmix64(base_seed ^ (0xA24BAED4963EE407ull * (uint64_t)(game_index + 1)));
}

static int or_timeout_thresh = OR_TIMEOUT_THRESH, or_win_score = OR_WIN_SCORE;

void or_set_limits(int timeout_thresh, int win_score) {
  or_timeout_thresh = timeout_thresh > 0 ? timeout_thresh : OR_TIMEOUT_THRESH;
  or_win_score = win_score > 0 ? win_score : OR_WIN_SCORE;
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

void or_env_reset(or_pong_state *s, uint64_t game_seed, int one_player) {
  memset(s, 0, sizeof(*s));
  s->seed = game_seed;
  s->one_player = one_player;
  s->lpy = 72;
  s->rpy = 72;
  s->ball_x = 79;
  s->ball_y = 78;
  s->ball_visible = 0;
  s->serve_timer = OR_SERVE_DELAY;
  s->serve_dir = 1; /* first serve travels toward the right paddle (the genome) */
}

int or_env_done(const or_pong_state *s) {
  return s->score1 >= OR_DONE_SCORE || s->score2 >= OR_DONE_SCORE;
}

static void spawn_ball(or_pong_state *s) {
  static const int vy_tab[4] = {-2, -1, 1, 2};
  uint64_t r = or_splitmix64(s->seed ^ ((uint64_t)(s->point + 1) * 0xD1B54A32D192ED03ull));
  s->ball_x = 79;
  s->ball_y = 40 + (int)(r % 77u);
  s->ball_vy = vy_tab[(r >> 32) & 3u];
  s->ball_vx = s->serve_dir * OR_BALL_VX0;
  s->hits = 0;
  s->ball_visible = 1;
  s->point += 1;
}

static int move_paddle(int y, int up, int dn, int speed) {
  if (up && !dn) y -= speed;
  else if (dn && !up) y += speed;
  return clampi(y, OR_PADDLE_Y_MIN, OR_PADDLE_Y_MAX);
}

void or_env_step(or_pong_state *s, int r_up, int r_dn, int l_up, int l_dn) {
  /* 1. paddles (the action was decided on the previous frame: main.py:77,91-92) */
  s->rpy = move_paddle(s->rpy, r_up, r_dn, OR_PADDLE_SPEED);
  if (s->one_player) {
    /* stand-in for the ROM's built-in opponent (1-player env, main.py:40) */
    int up = 0, dn = 0;
    if (s->ball_visible) {
      int bc2 = 2 * s->ball_y + OR_BALL_H - 1;
      int pc2 = 2 * s->lpy + OR_PADDLE_H - 1;
      if (bc2 < pc2 - 4) up = 1;
      else if (bc2 > pc2 + 4) dn = 1;
    }
    s->lpy = move_paddle(s->lpy, up, dn, OR_CPU_SPEED);
  } else {
    s->lpy = move_paddle(s->lpy, l_up, l_dn, OR_PADDLE_SPEED);
  }

  /* 2. ball */
  if (!s->ball_visible) {
    if (s->serve_timer > 0) s->serve_timer -= 1;
    if (s->serve_timer == 0 && !or_env_done(s)) spawn_ball(s);
    return;
  }
  int x = s->ball_x, y = s->ball_y;
  int nx = x + s->ball_vx, ny = y + s->ball_vy;
  int vy = s->ball_vy;
  const int ymax = OR_FIELD_H - OR_BALL_H; /* 156 */
  if (ny < 0) {
    ny = -ny;
    vy = -vy;
  } else if (ny > ymax) {
    ny = 2 * ymax - ny;
    vy = -vy;
  }
  const int lface = OR_LEFT_PADDLE_X + OR_PADDLE_W; /* 20: first column right of the left paddle */
  const int rface = OR_RIGHT_PADDLE_X;              /* 140 */
  int vx = s->ball_vx;
  /* A visible ball never enters a paddle's columns: crossing a paddle face
   * is either a bounce (rows overlap) or a miss, which scores at once.  So
   * the rendered frame never has overlapping objects and find_stuff's
   * centroids equal the analytic ones (tests/golden: centroids). */
  if (vx < 0 && nx <= lface - 1) {
    if (ny <= s->lpy + OR_PADDLE_H - 1 && ny + OR_BALL_H - 1 >= s->lpy) {
      s->hits += 1;
      int mag = OR_BALL_VX0 + s->hits / 4;
      if (mag > OR_BALL_VX_MAX) mag = OR_BALL_VX_MAX;
      nx = lface;
      vx = mag;
      vy = (2 * (ny - s->lpy) - 12) / 6; /* C division truncates toward zero */
    } else { /* miss on the left: the right player (score2) scores */
      s->score2 += 1;
      s->ball_visible = 0;
      s->serve_timer = OR_SERVE_DELAY;
      s->serve_dir = -1;
      return;
    }
  } else if (vx > 0 && nx + OR_BALL_W - 1 >= rface) {
    if (ny <= s->rpy + OR_PADDLE_H - 1 && ny + OR_BALL_H - 1 >= s->rpy) {
      s->hits += 1;
      int mag = OR_BALL_VX0 + s->hits / 4;
      if (mag > OR_BALL_VX_MAX) mag = OR_BALL_VX_MAX;
      nx = rface - OR_BALL_W;
      vx = -mag;
      vy = (2 * (ny - s->rpy) - 12) / 6;
    } else { /* miss on the right: the left player (score1) scores */
      s->score1 += 1;
      s->ball_visible = 0;
      s->serve_timer = OR_SERVE_DELAY;
      s->serve_dir = 1;
      return;
    }
  }
  s->ball_x = nx;
  s->ball_y = ny;
  s->ball_vx = vx;
  s->ball_vy = vy;
}

/* Doubled centroid row of a paddle clipped to the playfield rows [0,160):
 * get_rect_quickly (utils.py:60-68) on the rendered rectangle. */
static int paddle_c2(int py) {
  int lo = py < 0 ? 0 : py;
  int hi = py + OR_PADDLE_H - 1;
  if (hi > OR_FIELD_H - 1) hi = OR_FIELD_H - 1;
  return lo + hi;
}

int or_gene_count(const or_net *net) {
  int b = net->bias ? 1 : 0, total = 0;
  for (int i = 0; i + 1 < net->n_nodes; ++i) total += (net->nodes[i] + b) * net->nodes[i + 1];
  return total; /* utils.calculate_gene_size, utils.py:128-136 */
}

/* Row j of y = W @ x as numpy computes it (numpy_nn.py:127 np.dot(w, column)).
 * numpy hands a C-contiguous float64 matrix times a vector to cblas_dgemv
 * (RowMajor, NoTrans), which OpenBLAS runs as dgemv_t over the transposed view:
 * each output is a dot product of length m, taken in blocks of at most 2048
 * elements (the last block m2 = (m & 2047) - (m & 3), the m & 3 trailing
 * elements after all blocks).  Within a block the kernel depends on the output's
 * position among the n outputs (dgemv_t_4.c: 4 outputs at a time, then 2, then 1):
 *   kind 0 (j < 4*(n/4)): 4 partial sums i mod 4, fused multiply-add,
 *                         block = (s0 + s2) + (s1 + s3);
 *   kind 1 (next 2 if n & 2): 2 partial sums i mod 2, product rounded then added,
 *                         block = s0 + s1;
 *   kind 2 (last if n & 1): 4 partial sums i mod 4, product rounded then added,
 *                         block = (s0 + s2) + (s1 + s3);
 * y accumulates the blocks (y + block); then the tail: 1 element y = fma(a, x, y);
 * 2: y + fma(a0, x0, a1 x1); 3: y + fma(a2, x2, fma(a0, x0, a1 x1)).  That is the
 * x86-64 AVX2/FMA kernel numpy's OpenBLAS (0.3.29, DYNAMIC_ARCH) selects on
 * Haswell-class and later cores, checked against np.dot in tests/test_blas_order.py. */
double or_blas_dot(const double *a, const double *x, int m, int j, int n) {
  const int kind = j < 4 * (n >> 2) ? 0 : ((n & 2) && j < 4 * (n >> 2) + 2) ? 1 : 2;
  const int m3 = m & 3, m2 = (m & 2047) - m3;
  int m1 = m & ~3, nb = 2048, start = 0;
  double y = 0.0;
  while (nb == 2048) {
    m1 -= nb;
    if (m1 < 0) {
      if (m2 == 0) break;
      nb = m2;
    }
    double s[4] = {0.0, 0.0, 0.0, 0.0}, blk;
    const double *ab = a + start, *xb = x + start;
    if (kind == 0) {
      for (int i = 0; i < nb; ++i) s[i & 3] = fma(ab[i], xb[i], s[i & 3]);
      blk = (s[0] + s[2]) + (s[1] + s[3]);
    } else if (kind == 1) {
      for (int i = 0; i < nb; ++i) {
        const double p = ab[i] * xb[i];
        s[i & 1] = s[i & 1] + p;
      }
      blk = s[0] + s[1];
    } else {
      for (int i = 0; i < nb; ++i) {
        const double p = ab[i] * xb[i];
        s[i & 3] = s[i & 3] + p;
      }
      blk = (s[0] + s[2]) + (s[1] + s[3]);
    }
    y = y + blk;
    start += nb;
  }
  const double *at = a + start, *xt = x + start;
  if (m3 == 1) {
    y = fma(at[0], xt[0], y);
  } else if (m3 == 2) {
    const double p1 = at[1] * xt[1];
    y = y + fma(at[0], xt[0], p1);
  } else if (m3 == 3) {
    const double p1 = at[1] * xt[1];
    y = y + fma(at[2], xt[2], fma(at[0], xt[0], p1));
  }
  return y;
}

void or_blas_gemv(const double *w, int n, int m, const double *x, double *y) {
  for (int j = 0; j < n; ++j) y[j] = or_blas_dot(w + (long)j * m, x, m, j, n);
}

int or_nn_run(const double *genes, const or_net *net, const double *x, double *out_act) {
  double buf0[OR_MAX_WIDTH + 1], buf1[OR_MAX_WIDTH + 1];
  double *cur = buf0, *nxt = buf1;
  const int b = net->bias ? 1 : 0;
  const int n_in = net->nodes[0];
  for (int i = 0; i < n_in; ++i) cur[i] = x[i];
  if (b) cur[n_in] = 1.0;
  long off = 0;
  for (int l = 0; l + 1 < net->n_nodes; ++l) {
    const int nin = net->nodes[l], nout = net->nodes[l + 1], cols = nin + b;
    for (int j = 0; j < nout; ++j) {
      const double *w = genes + off + (long)j * cols; /* row-major (out, in+bias) numpy_nn.py:63 */
      const double z = or_blas_dot(w, cur, cols, j, nout); /* np.dot(w, column), numpy_nn.py:127 */
      nxt[j] = 1.0 / (1.0 + pow(M_E, -z)); /* 1 / (1 + np.e ** -x), numpy_nn.py:22-23 */
    }
    if (b) nxt[nout] = 1.0;
    off += (long)cols * nout;
    double *t = cur;
    cur = nxt;
    nxt = t;
  }
  const int n_out = net->nodes[net->n_nodes - 1];
  int best = 0; /* np.argmax: the first NaN if any, else the first maximum */
  for (int j = 1; j < n_out && !isnan(cur[best]); ++j)
    if (isnan(cur[j]) || cur[j] > cur[best]) best = j;
  if (out_act)
    for (int j = 0; j < n_out; ++j) out_act[j] = cur[j];
  return best;
}

/* action codes: 0 = [0,0], 1 = [1,0] (up), 2 = [0,1] (down) */
static int index_to_code(int idx) { return idx == 0 ? 1 : (idx == 1 ? 2 : 0); }

static int hardcoded(const double *x) { /* HardcodedAi.run dumb_ais.py:2-8 */
  if (x[1] < x[4]) return 1;
  if (x[1] > x[4]) return 2;
  return 0;
}

static int clamp_action(int c2, int code) { /* keep_within_game_bounds_please utils.py:71-77 */
  double y = 0.5 * (double)c2;
  if (y < 16.0) return 2;
  if (y > (double)(OR_FIELD_H) - 16.0) return 1;
  return code;
}

/* perform_episode's return value (main.py:108-112, calculate_reward utils.py:104-109) */
static double episode_reward(const or_pong_state *s, double total, double mult, int *zero_division) {
  *zero_division = 0;
  if (s->score1 == s->score2) return 0.0; /* main.py:109-110 */
  if (total == 0.0) {
    *zero_division = 1; /* utils.py:106-108 would raise ZeroDivisionError */
    return NAN;
  }
  double diff = (double)(s->score2 - s->score1);
  double scaled = total / 100.0;
  double bonus = (double)s->score2 * mult;
  return (diff + bonus) / scaled;
}

/* One game slot.  horizon <= 0: one perform_episode (main.py:69-112).
 * horizon T > 0: SURVEY 8(d)'s fixed-horizon measurement mode (pong_ga.h
 * pg_eval_args.horizon): exactly T frames; an episode that terminates before
 * frame T is scored and the env auto-resets (the serve sequence continues:
 * the point counter is kept), the partial last episode is dropped.  Result:
 * reward = the completed episodes' rewards summed in order, score1/score2 =
 * the points of all episodes, frames = T, total_frames = completed episodes. */
void or_play_slot(const double *genes, const or_net *net, int opp_kind, const double *opp_genes, double mult,
                  uint64_t game_seed, int horizon, or_game_result *out, uint8_t *trace, int trace_cap) {
  or_pong_state s;
  or_env_reset(&s, game_seed, opp_kind == OR_OPP_ROM_CPU);
  int act_r = 0, act_l = 0;
  double timeout = 0.0, total = 0.0;
  int have_last_score = 0, last1 = 0, last2 = 0;
  int have_last_ball = 0, lby2 = 0, lbx2 = 0;
  int frames = 0;
  double h_reward = 0.0;
  int h_eps = 0, h_s1 = 0, h_s2 = 0, h_zd = 0;
  for (;;) {
    or_env_step(&s, act_r == 1, act_r == 2, act_l == 1, act_l == 2);
    frames += 1;
    const int vis = s.ball_visible;
    const int by2 = 2 * s.ball_y + OR_BALL_H - 1, bx2 = 2 * s.ball_x + OR_BALL_W - 1;
    const int lc2 = paddle_c2(s.lpy), rc2 = paddle_c2(s.rpy);
    int left = 0, right = 0;
    /* get_actions main.py:138-154.  Both paddles are always (partly) visible
     * in this physics, so the get_random_action defaults (utils.py:112-113)
     * are never the returned action. */
    if (vis) {
      const int pby2 = have_last_ball ? lby2 : by2, pbx2 = have_last_ball ? lbx2 : bx2;
      double xr[6], xl[6];
      /* inference utils.py:139-153: [bx, by, lbx, lby, me, enemy] / 160 */
      xr[0] = (0.5 * bx2) / 160.0;
      xr[1] = (0.5 * by2) / 160.0;
      xr[2] = (0.5 * pbx2) / 160.0;
      xr[3] = (0.5 * pby2) / 160.0;
      xr[4] = (0.5 * rc2) / 160.0;
      xr[5] = (0.5 * lc2) / 160.0;
      /* left side sees the x axis flipped: GAME_WIDTH - x, main.py:146-147 */
      xl[0] = (160.0 - 0.5 * bx2) / 160.0;
      xl[1] = (0.5 * by2) / 160.0;
      xl[2] = (160.0 - 0.5 * pbx2) / 160.0;
      xl[3] = (0.5 * pby2) / 160.0;
      xl[4] = (0.5 * lc2) / 160.0;
      xl[5] = (0.5 * rc2) / 160.0;
      switch (opp_kind) {
        case OR_OPP_HARDCODED:
        case OR_OPP_ROM_CPU: left = hardcoded(xl); break;
        case OR_OPP_SCORE: left = (s.score1 <= s.score2) ? hardcoded(xl) : 0; break;
        default: left = index_to_code(or_nn_run(opp_genes, net, xl, NULL)); break;
      }
      right = index_to_code(or_nn_run(genes, net, xr, NULL));
    }
    have_last_ball = vis;
    lby2 = by2;
    lbx2 = bx2;
    left = clamp_action(lc2, left);
    right = clamp_action(rc2, right);
    act_l = left;
    act_r = right;
    if (trace && frames <= trace_cap)
      trace[frames - 1] = (uint8_t)(right | (left << 2) | (vis << 4));
    /* calculate_timeout_and_frames main.py:128-135 */
    if (have_last_score) {
      if (s.score1 == last1 && s.score2 == last2) {
        timeout += 1.0;
      } else {
        total += timeout;
        timeout = 0.0;
      }
    }
    have_last_score = 1;
    last1 = s.score1;
    last2 = s.score2;
    /* termination main.py:102-107 */
    const int ep_end = s.score1 >= or_win_score || s.score2 >= or_win_score || or_env_done(&s) ||
                       timeout > (double)or_timeout_thresh;
    if (horizon <= 0) {
      if (ep_end) break;
      continue;
    }
    if (ep_end) { /* score the episode, then auto-reset the slot */
      int zd = 0;
      h_reward += episode_reward(&s, total, mult, &zd);
      h_zd |= zd;
      h_eps += 1;
      h_s1 += s.score1;
      h_s2 += s.score2;
      if (frames >= horizon) break;
      const int point = s.point;
      or_env_reset(&s, game_seed, opp_kind == OR_OPP_ROM_CPU);
      s.point = point;
      act_r = act_l = 0;
      timeout = total = 0.0;
      have_last_score = have_last_ball = 0;
      continue;
    }
    if (frames >= horizon) { /* the partial last episode: its points only */
      h_s1 += s.score1;
      h_s2 += s.score2;
      break;
    }
  }
  out->slow_decisions = 0;
  out->frames = frames;
  if (horizon > 0) {
    out->score1 = h_s1;
    out->score2 = h_s2;
    out->total_frames = (double)h_eps;
    out->reward = h_reward;
    out->zero_division = h_zd;
    return;
  }
  out->score1 = s.score1;
  out->score2 = s.score2;
  out->total_frames = total;
  out->reward = episode_reward(&s, total, mult, &out->zero_division);
}

void or_play_game(const double *genes, const or_net *net, int opp_kind,
                  const double *opp_genes, double mult, uint64_t game_seed,
                  or_game_result *out, uint8_t *trace, int trace_cap) {
  or_play_slot(genes, net, opp_kind, opp_genes, mult, game_seed, 0, out, trace, trace_cap);
}

int or_eval_population(int n, int n_games, const double *genomes, int64_t stride,
                       const double *opponents, int64_t opp_stride,
                       const int32_t *kind, const int32_t *opp_index,
                       const double *mult, const or_net *net, uint64_t base_seed,
                       double *fitness, double *rewards, int32_t *scores,
                       int32_t *frames, double *total_frames, int32_t *status,
                       int n_threads) {
  return or_eval_population_h(n, n_games, genomes, stride, opponents, opp_stride, kind, opp_index, mult, net,
                              base_seed, 0, fitness, rewards, scores, frames, total_frames, status, n_threads);
}

int or_eval_population_h(int n, int n_games, const double *genomes, int64_t stride,
                         const double *opponents, int64_t opp_stride,
                         const int32_t *kind, const int32_t *opp_index,
                         const double *mult, const or_net *net, uint64_t base_seed, int horizon,
                         double *fitness, double *rewards, int32_t *scores,
                         int32_t *frames, double *total_frames, int32_t *status,
                         int n_threads) {
  int first_err = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads > 0 ? n_threads : 1) if (n_threads > 1)
#endif
  for (int i = 0; i < n; ++i) {
    double sum = 0.0;
    int err = 0;
    for (int g = 0; g < n_games; ++g) {
      const long k = (long)i * n_games + g;
      const double *opp = NULL;
      if (kind[k] == OR_OPP_NN) opp = opponents + (long)opp_index[k] * opp_stride;
      or_game_result r;
      or_play_slot(genomes + (long)i * stride, net, kind[k], opp, mult[k],
                   or_game_seed(base_seed, g), horizon, &r, NULL, 0);
      if (rewards) rewards[k] = r.reward;
      if (scores) {
        scores[2 * k] = r.score1;
        scores[2 * k + 1] = r.score2;
      }
      if (frames) frames[k] = r.frames;
      if (total_frames) total_frames[k] = r.total_frames;
      err |= r.zero_division;
      sum += r.reward; /* sum(all_rewards), main.py:65 */
    }
    fitness[i] = sum / (double)n_games; /* main.py:65-66 */
    if (status) status[i] = err;
    if (err) {
#ifdef _OPENMP
#pragma omp critical
#endif
      if (first_err == 0 || i + 1 < first_err) first_err = i + 1;
    }
  }
  return first_err;
}

/* ------------------------------------------------------------ pixel path -- */
static const uint8_t OR_COLOURS[4][3] = {{144, 72, 17},    /* BG_COLOUR        config.py */
                                        {236, 236, 236},  /* BALL_COLOUR                */
                                        {213, 130, 74},   /* LEFT_GUY_COLOUR            */
                                        {92, 186, 92}};   /* RIGHT_GUY_COLOUR           */

static void paint(uint8_t *frame, int r0, int r1, int c0, int c1, int colour) { /* rows [r0,r1), cols [c0,c1) */
  for (int r = r0; r < r1; ++r)
    for (int c = c0; c < c1; ++c)
      for (int ch = 0; ch < 3; ++ch) frame[(r * 160 + c) * 3 + ch] = OR_COLOURS[colour][ch];
}

void or_render(const or_pong_state *s, uint8_t *frame) {
  const int top = 34; /* GAME_TOP */
  paint(frame, 0, 210, 0, 160, 0);
  paint(frame, 24, 34, 0, 160, 1);
  paint(frame, 194, 210, 0, 160, 1);
  const int pys[2] = {s->lpy, s->rpy}, xs[2] = {OR_LEFT_PADDLE_X, OR_RIGHT_PADDLE_X};
  for (int k = 0; k < 2; ++k) {
    const int lo = pys[k] < 0 ? 0 : pys[k];
    const int hi = pys[k] + OR_PADDLE_H - 1 > OR_FIELD_H - 1 ? OR_FIELD_H - 1 : pys[k] + OR_PADDLE_H - 1;
    paint(frame, top + lo, top + hi + 1, xs[k], xs[k] + OR_PADDLE_W, 2 + k);
  }
  if (s->ball_visible) paint(frame, top + s->ball_y, top + s->ball_y + OR_BALL_H, s->ball_x, s->ball_x + OR_BALL_W, 1);
}

void or_find_stuff(const uint8_t *frame, double *out) {
  /* np.average(np.argwhere(crop == colour)[:, :-1], axis=0): one (row, col)
   * per matching CHANNEL; integer sums are exact, one rounding in the mean */
  for (int k = 0; k < 3; ++k) {
    long long n = 0, rs = 0, cs = 0;
    for (int r = 0; r < 160; ++r)
      for (int c = 0; c < 160; ++c)
        for (int ch = 0; ch < 3; ++ch)
          if (frame[((34 + r) * 160 + c) * 3 + ch] == OR_COLOURS[k + 1][ch]) {
            n += 1;
            rs += r;
            cs += c;
          }
    out[2 * k] = n ? (double)rs / (double)n : NAN;
    out[2 * k + 1] = n ? (double)cs / (double)n : NAN;
  }
}
