// pg_gen.hip -- the device work of one eaSimple generation around the
// evaluation (DeviceGA, pong_amd/evolve.py; the reference's step is DEAP's
// eaSimple, main.py:165-170, with the operators ga.py:89-94): few launches,
// one host sync before the hall-of-fame scan and one after it.
//
//   pg_ga_scatter_fitness   evaluation results -> the shard's row order, and
//                           each played row's longest game (evaluation order)
//   pg_ga_merge_fitness     clones keep their parent's fitness (varAnd), the
//                           logbook statistics (main.py:158-162), NaN check
//                           (calculate_reward's ZeroDivisionError,
//                           utils.py:106-108) and the hall-of-fame candidates
//                           (fitness > the full hall's worst), ascending
//   pg_ga_select_ranked     selTournament (ga.py:94) by rank sampling, with
//                           its fitness sort inside (rocPRIM)
//   pg_ga_inherit           what an offspring inherits from its parent
//   pg_ga_order             the shard's evaluation order: invalid_ind first,
//                           longest lineage game first
//   pg_hof_prepare_cand     HallOfFame.update's scan input for k candidates:
//                           hashes, (fitness, age) ranks by a candidate-only
//                           sort and binary searches into the ordered
//                           members, dense similarity classes by hash tables
//   pg_hof_commit           the new hall: rows, hashes and fitness in one pass
#include <hip/hip_runtime.h>

#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>

#include "pg_eval.hpp"


namespace pg {
namespace {

constexpr int kT = 256;             // threads per block
constexpr int kChunk = 8 * kT;      // merge: elements per block
inline unsigned blocks(long n, int per = kT) { return (unsigned)((n + per - 1) / per); }
inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// ------------------------------------------------------------ scatter ----
__global__ void k_scatter_fitness(pg_scatter_args a) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= a.n) return;
  const int played = a.n_active ? __builtin_amdgcn_readfirstlane(*a.n_active) : a.n;
  const int row = a.rows ? a.rows[i] : a.row_lo + i;
  const bool p = i < played;
  a.shard_fitness[row - a.row_lo] = p ? a.fitness[i] : 0.0;
  if (p && a.lineage) {
    int m = 0;
    for (int g = 0; g < a.n_games; ++g) m = max(m, a.frames[(long)i * a.n_games + g]);
    a.lineage[row] = (float)m;
  }
}

// -------------------------------------------------------------- merge ----
// Per-block partials: (count, mean, M2) by Chan's parallel update, min, max,
// NaN flag, nevals, candidates.  Every reduction runs in a fixed order, so the
// statistics are reproducible bit for bit.
struct Part {
  double n, mean, m2, mn, mx;
  int32_t nan, nevals, cand, pad;
};

__device__ inline void chan(double &n, double &mean, double &m2, double nb, double meanb, double m2b) {
  if (nb == 0.0) return;
  if (n == 0.0) {
    n = nb, mean = meanb, m2 = m2b;
    return;
  }
  const double t = n + nb, d = meanb - mean;
  mean += d * (nb / t);
  m2 += m2b + d * d * (n * nb / t);
  n = t;
}

__device__ inline void part_merge(Part &x, const Part &y) {
  chan(x.n, x.mean, x.m2, y.n, y.mean, y.m2);
  x.mn = fmin(x.mn, y.mn);
  x.mx = fmax(x.mx, y.mx);
  x.nan |= y.nan;
  x.nevals += y.nevals;
  x.cand += y.cand;
}

__device__ inline bool is_cand(const pg_merge_args &a, double f) { return !a.filter || f > a.worst; }

__device__ inline double merged(const pg_merge_args &a, int i) {
  return (!a.invalid || a.invalid[i]) ? a.fitness[i] : a.inherited[i];
}

__global__ __launch_bounds__(kT) void k_merge_partials(pg_merge_args a, Part *parts) {
  __shared__ Part sh[kT];
  Part p{0.0, 0.0, 0.0, __builtin_inf(), -__builtin_inf(), 0, 0, 0, 0};
  const long base = (long)blockIdx.x * kChunk;
  for (int e = 0; e < kChunk / kT; ++e) {
    const long i = base + (long)e * kT + threadIdx.x;
    if (i >= a.pop_n) break;
    const double f = merged(a, (int)i);
    a.new_fitness[i] = f;
    p.nevals += (!a.invalid || a.invalid[i]) ? 1 : 0;
    if (f != f) {
      p.nan = 1;
      continue;
    }
    chan(p.n, p.mean, p.m2, 1.0, f, 0.0);
    p.mn = fmin(p.mn, f);
    p.mx = fmax(p.mx, f);
    p.cand += is_cand(a, f) ? 1 : 0;
  }
  sh[threadIdx.x] = p;
  __syncthreads();
  for (int s = kT / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) part_merge(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) parts[blockIdx.x] = sh[0];
}

// one block: the summary, and each block's first candidate slot
__global__ __launch_bounds__(kT) void k_merge_finish(pg_merge_args a, const Part *parts, int nb, int32_t *offsets) {
  if (threadIdx.x != 0) return;
  Part t{0.0, 0.0, 0.0, __builtin_inf(), -__builtin_inf(), 0, 0, 0, 0};
  for (int b = 0; b < nb; ++b) {
    offsets[b] = t.cand;
    part_merge(t, parts[b]);
  }
  double *s = a.summary;
  s[0] = t.nan ? 1.0 : 0.0;
  s[1] = t.n > 0.0 ? t.mean : __builtin_nan("");
  s[2] = t.n > 0.0 ? sqrt(t.m2 / t.n) : __builtin_nan("");  // population std (np.std, ddof 0)
  s[3] = t.n > 0.0 ? t.mn : __builtin_nan("");
  s[4] = t.n > 0.0 ? t.mx : __builtin_nan("");
  s[5] = (double)t.nevals;
  s[6] = (double)t.cand;
  s[7] = 0.0;
}

// candidates in ascending row order: block-local exclusive scan of the flags
__global__ __launch_bounds__(kT) void k_merge_compact(pg_merge_args a, const int32_t *offsets) {
  __shared__ int32_t cnt[kT];
  const long base = (long)blockIdx.x * kChunk + (long)threadIdx.x * (kChunk / kT);
  bool fl[kChunk / kT];
  int c = 0;
  for (int e = 0; e < kChunk / kT; ++e) {
    const long i = base + e;
    const double f = i < a.pop_n ? a.new_fitness[i] : 0.0;
    fl[e] = i < a.pop_n && f == f && is_cand(a, f);
    c += fl[e] ? 1 : 0;
  }
  cnt[threadIdx.x] = c;
  __syncthreads();
  // inclusive Hillis-Steele scan over the block's threads
  for (int s = 1; s < kT; s <<= 1) {
    const int v = (int)threadIdx.x >= s ? cnt[threadIdx.x - s] : 0;
    __syncthreads();
    cnt[threadIdx.x] += v;
    __syncthreads();
  }
  int at = offsets[blockIdx.x] + cnt[threadIdx.x] - c;
  for (int e = 0; e < kChunk / kT; ++e) {
    if (!fl[e]) continue;
    const long i = base + e;
    a.cand[at] = (int32_t)i;
    a.cand_fitness[at] = a.new_fitness[i];
    ++at;
  }
}

// -------------------------------------------------------------- order ----
__global__ void k_order_keys(int n, int lo, const uint8_t *invalid, const float *lineage, int by_length,
                             uint32_t *keys, int32_t *vals, int32_t *count) {
  const int i = blockIdx.x * kT + threadIdx.x;
  const bool inv = i < n && (!invalid || invalid[lo + i]);
  if (i < n) {
    uint32_t k = 0xFFFFFFFFu;
    if (inv) {
      const float L = lineage && by_length ? lineage[lo + i] : 0.0f;
      const uint32_t li = L > 0.0f ? (L < 4.0e9f ? (uint32_t)L : 0xFFFFFFF0u) : 0u;
      k = 0xFFFFFFFEu - (li < 0xFFFFFFFEu ? li : 0xFFFFFFFEu);
    }
    keys[i] = k;
    vals[i] = lo + i;
  }
  // integer count: any order, same total
  const unsigned long long b = __ballot(inv);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (int32_t)__popcll(b));
}

// -------------------------------------------------------------- inherit --
__global__ void k_inherit(const int32_t *chosen, int n, const double *fitness, double *inherited,
                          const float *lineage_in, float *lineage_out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const int c = chosen[i];
  if (inherited) inherited[i] = fitness[c];
  if (lineage_out) lineage_out[i] = lineage_in[c];
}

// ---------------------------------------------------- hall-of-fame prep --
// Open-addressing tables keyed by the 64-bit row hash, value = the smallest
// index holding it (atomicMin: the same result in any insertion order).  The
// key 0xFFFF...FF marks an empty slot; a genuine hash of that value lives in
// the extra slot at [cap].
struct Slot {
  unsigned long long key;
  unsigned int idx;
  unsigned int pad;
};
constexpr unsigned long long kEmpty = ~0ull;

__device__ inline unsigned mix_slot(unsigned long long h, unsigned cap) {
  return (unsigned)((h * 0x9E3779B97F4A7C15ull) >> 32) & (cap - 1);
}

__device__ inline void table_insert(Slot *t, unsigned cap, unsigned long long h, unsigned idx) {
  if (h == kEmpty) {
    atomicMin(&t[cap].idx, idx);
    return;
  }
  unsigned s = mix_slot(h, cap);
  for (;;) {
    const unsigned long long old = atomicCAS(&t[s].key, kEmpty, h);
    if (old == kEmpty || old == h) {
      atomicMin(&t[s].idx, idx);
      return;
    }
    s = (s + 1) & (cap - 1);
  }
}

__device__ inline int table_find(const Slot *t, unsigned cap, unsigned long long h) {
  if (h == kEmpty) return t[cap].idx == 0xFFFFFFFFu ? -1 : (int)t[cap].idx;
  unsigned s = mix_slot(h, cap);
  for (;;) {
    const unsigned long long k = t[s].key;
    if (k == h) return (int)t[s].idx;
    if (k == kEmpty) return -1;
    s = (s + 1) & (cap - 1);
  }
}

__global__ void k_hof_insert(const uint64_t *hof_hash, int hn, Slot *mt, unsigned mcap, const uint64_t *cand_hash,
                             int k, Slot *ct, unsigned ccap) {
  const int e = blockIdx.x * kT + threadIdx.x;
  if (e < hn) {
    table_insert(mt, mcap, hof_hash[e], (unsigned)e);
  } else if (e < hn + k) {
    table_insert(ct, ccap, cand_hash[e - hn], (unsigned)(e - hn));
  }
}

// The two searches of k_hof_rank_pack, as first-false of a monotone
// predicate over a sorted array (true on a prefix).  Every block stages a
// sample of each array (every s-th element, <= kSamples of them) in LDS; the
// search runs over the sample, then counts the predicate over the s - 1
// elements of the one window left -- independent loads, where a binary search
// over global memory is ~14 dependent ones (this kernel shares the device
// with the side stream's vary and records, and its slowest thread sets it)
constexpr int kSamples = 2048;

__device__ inline int sample_stride(int len) { return len > kSamples ? (len + kSamples - 1) / kSamples : 1; }

__device__ inline void stage_samples(double *sh, const double *a, int len, int st) {
  const int ns = (len + st - 1) / st;
  for (int i = threadIdx.x; i < ns; i += kT) sh[i] = a[(long)i * st];
}

// first index m of a[0, len) whose pred(a[m]) is false (len if none)
template <typename Pred>
__device__ inline int first_false(const double *sh, const double *a, int len, int st, Pred pred) {
  const int ns = (len + st - 1) / st;
  int lo = 0, hi = ns;  // first sample whose predicate is false
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (pred(sh[m])) lo = m + 1; else hi = m;
  }
  if (st == 1 || lo == 0) return lo * st < len ? lo * st : len;
  // the answer lies in ((lo - 1) * st, min(lo * st, len)]
  const int w0 = (lo - 1) * st + 1, w1 = lo * st < len ? lo * st : len;
  int c = 0;
  for (int i = w0; i < w1; ++i) c += pred(a[i]) ? 1 : 0;
  return w0 + c;
}

// rank (ascending (fitness, age); members older than every candidate) and
// dense class of entry e, packed as pg_hof_rank_classes does
__global__ __launch_bounds__(256) void k_hof_rank_pack(const double *hof_fitness, const uint64_t *hof_hash, int hn,
                                                       const double *cand_fitness, const uint64_t *cand_hash, int k,
                                                       const double *sorted_fit, const int32_t *sorted_idx,
                                                       const Slot *mt, unsigned mcap, const Slot *ct, unsigned ccap,
                                                       int64_t *packed) {
  __shared__ double sh_cand[kSamples], sh_hof[kSamples];
  const int e = blockIdx.x * kT + threadIdx.x;
  const int n = hn + k;
  const int st_c = sample_stride(k), st_h = sample_stride(hn);
  // (block-uniform: which searches this block's entries run)
  const int b0 = blockIdx.x * kT, b1 = b0 + kT;
  if (b0 < hn) stage_samples(sh_cand, sorted_fit, k, st_c);
  if (b1 > hn) stage_samples(sh_hof, hof_fitness, hn, st_h);
  __syncthreads();
  if (e < k) packed[n + e] = __double_as_longlong(cand_fitness[e]);
  if (e >= n) return;
  int rank, cls;
  if (e < hn) {
    const double f = hof_fitness[e];
    // candidates strictly below f (equal ones are younger: above)
    const int lo = first_false(sh_cand, sorted_fit, k, st_c, [f](double x) { return x < f; });
    rank = (hn - 1 - e) + lo;
    cls = table_find(mt, mcap, hof_hash[e]);
  } else {
    // sorted slot s of this candidate: entries e-hn are scattered by the sort,
    // so this thread handles sorted slot s = e - hn instead
    const int s = e - hn;
    const int j = sorted_idx[s];
    const double f = sorted_fit[s];
    // members with fitness <= f: items order is descending, so count those > f
    const int lo = first_false(sh_hof, hof_fitness, hn, st_h, [f](double x) { return x > f; });
    rank = s + (hn - lo);
    const int mm = table_find(mt, mcap, cand_hash[j]);
    cls = mm >= 0 ? mm : hn + table_find(ct, ccap, cand_hash[j]);
    packed[hn + j] = (int64_t)(uint32_t)rank | ((int64_t)cls << 32);
    return;
  }
  packed[e] = (int64_t)(uint32_t)rank | ((int64_t)cls << 32);
}

unsigned table_cap(int n) {
  unsigned c = 64;
  while (c < 2u * (unsigned)(n > 0 ? n : 1)) c <<= 1;
  return c;
}

struct CandLayout {
  size_t mt, ct, sort_keys, sort_vals, sort_temp, total, temp_bytes;
  unsigned mcap, ccap;
};

int32_t cand_layout(int hn, int k, CandLayout *L) {
  size_t tb = 0;
  if (rocprim::radix_sort_pairs(nullptr, tb, (const double *)nullptr, (double *)nullptr, (const int32_t *)nullptr,
                                (int32_t *)nullptr, (unsigned)(k > 0 ? k : 1)) != hipSuccess)
    return fail(PG_ERR_HIP, "hof_prepare_cand: rocPRIM storage query failed");
  L->mcap = table_cap(hn);
  L->ccap = table_cap(k);
  size_t off = 0;
  auto take = [&](size_t b) {
    const size_t at = off;
    off += align_up(b);
    return at;
  };
  L->mt = take((size_t)(L->mcap + 1) * sizeof(Slot));
  L->ct = take((size_t)(L->ccap + 1) * sizeof(Slot));
  const size_t kk = (size_t)(k > 0 ? k : 1);
  L->sort_keys = take(kk * 8 * 2);  // normalised keys in, sorted out
  L->sort_vals = take(kk * 4 * 2);  // iota in, order out
  L->temp_bytes = tb > 0 ? tb : 1;
  L->sort_temp = take(L->temp_bytes);
  L->total = off;
  return PG_OK;
}

__global__ void k_iota(int32_t *v, int n) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i < n) v[i] = i;
}

// sort keys of the candidates: -0.0 as +0.0, so the radix order agrees with
// the == of HallOfFame's comparisons (equal fitness: age decides)
__global__ void k_cand_keys(const double *f, int k, double *keys, int32_t *iota) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= k) return;
  keys[i] = f[i] + 0.0;
  iota[i] = i;
}

// one wave per hall position, four per block, striding over the positions:
// the in-place commit copies only the entering candidates' rows, so most
// waves write two words -- a block per position was mostly launch cost
template <typename WT>
__global__ __launch_bounds__(256) void k_hof_commit(WT *dst, int64_t dst_stride, const WT *old_rows, int64_t old_stride,
                                                    const WT *rows, int64_t rows_stride, const int32_t *cand,
                                                    const int32_t *src, int m, int n_old, int64_t genes,
                                                    const uint64_t *old_hash, const uint64_t *cand_hash,
                                                    uint64_t *new_hash, const double *fit_in, double *new_fitness,
                                                    const int32_t *dst_slot) {
  const int lane = threadIdx.x & 63;
  for (int j = blockIdx.x * 4 + (threadIdx.x >> 6); j < m; j += gridDim.x * 4) {
    const int s = src[j];
    // (dst_slot: the hall in place -- a kept member's row is already in its slot)
    if (!dst_slot || s >= n_old) {
      const WT *from = s < n_old ? old_rows + (long)s * old_stride : rows + (long)cand[s - n_old] * rows_stride;
      WT *to = dst + (long)(dst_slot ? dst_slot[j] : j) * dst_stride;
      for (int64_t g = lane; g < genes; g += 64) to[g] = from[g];
    }
    if (lane == 0) {
      new_hash[j] = s < n_old ? old_hash[s] : cand_hash[s - n_old];
      new_fitness[j] = fit_in[j];
    }
  }
}

}  // namespace
}  // namespace pg

using namespace pg;

extern "C" {

int32_t pg_ga_scatter_fitness(const pg_scatter_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  if (a->n < 0 || a->n_games < 1 || a->row_lo < 0 || (a->n > 0 && (!a->fitness || !a->shard_fitness)) ||
      (a->n > 0 && a->lineage && !a->frames))
    return fail(PG_ERR_INVALID, "ga_scatter_fitness: bad sizes or NULL buffers");
  if (a->n == 0) return PG_OK;
  hipLaunchKernelGGL(k_scatter_fitness, dim3(blocks(a->n)), dim3(kT), 0, (hipStream_t)stream, *a);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

size_t pg_ga_merge_workspace_bytes(int32_t pop_n) {
  if (pop_n < 0) return 0;
  const size_t nb = blocks(pop_n > 0 ? pop_n : 1, kChunk);
  return align_up(nb * sizeof(Part)) + align_up(nb * sizeof(int32_t));
}

int32_t pg_ga_merge_fitness(const pg_merge_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  const int n = a->pop_n;
  if (n < 0 || !a->summary || (n > 0 && (!a->fitness || !a->new_fitness || !a->cand || !a->cand_fitness)) ||
      (n > 0 && a->invalid && !a->inherited))
    return fail(PG_ERR_INVALID, "ga_merge_fitness: bad sizes or NULL buffers");
  const size_t need = pg_ga_merge_workspace_bytes(n);
  if (!a->workspace || a->workspace_bytes < need)
    return fail(PG_ERR_INVALID, "ga_merge_fitness: workspace of %zu bytes needed", need);
  const unsigned nb = blocks(n > 0 ? n : 1, kChunk);
  Part *parts = (Part *)a->workspace;
  int32_t *offsets = (int32_t *)((char *)a->workspace + align_up(nb * sizeof(Part)));
  const hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_merge_partials, dim3(nb), dim3(kT), 0, s, *a, parts);
  hipLaunchKernelGGL(k_merge_finish, dim3(1), dim3(64), 0, s, *a, (const Part *)parts, (int)nb, offsets);
  hipLaunchKernelGGL(k_merge_compact, dim3(nb), dim3(kT), 0, s, *a, (const int32_t *)offsets);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

size_t pg_ga_select_workspace_bytes(int32_t n_pop) {
  if (n_pop < 0) return 0;
  const unsigned n = (unsigned)(n_pop > 0 ? n_pop : 1);
  size_t tb = 0;
  if (rocprim::radix_sort_pairs(nullptr, tb, (const double *)nullptr, (double *)nullptr, (const int32_t *)nullptr,
                                (int32_t *)nullptr, n) != hipSuccess)
    return 0;
  return align_up((size_t)n * 8) + 2 * align_up((size_t)n * 4) + align_up(tb > 0 ? tb : 1);
}

int32_t pg_ga_select_ranked(const pg_select_args *a, void *workspace, size_t workspace_bytes, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  if (a->n_pop < 1 || a->k < 0 || a->tournsize < 1 || !a->fitness || (a->k > 0 && !a->chosen))
    return fail(PG_ERR_INVALID, "ga_select_ranked: bad sizes or NULL buffers");
  const size_t need = pg_ga_select_workspace_bytes(a->n_pop);
  if (need == 0 || !workspace || workspace_bytes < need)
    return fail(PG_ERR_INVALID, "ga_select_ranked: workspace of %zu bytes needed", need);
  const unsigned n = (unsigned)a->n_pop;
  char *ws = (char *)workspace;
  double *sorted = (double *)ws;
  int32_t *iota = (int32_t *)(ws + align_up((size_t)n * 8));
  int32_t *order = (int32_t *)((char *)iota + align_up((size_t)n * 4));
  void *temp = (char *)order + align_up((size_t)n * 4);
  size_t tb = workspace_bytes - ((char *)temp - ws);
  const hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_iota, dim3(blocks(n)), dim3(kT), 0, s, iota, (int)n);
  // stable: equal fitness keeps row order (torch.sort(stable=True) before)
  PG_HIP(rocprim::radix_sort_pairs(temp, tb, a->fitness, sorted, iota, order, n, 0, 64, s));
  return pg_ga_select_tournament_ranked(a, sorted, order, stream);
}

int32_t pg_ga_inherit(const int32_t *chosen, int32_t n, const double *fitness, double *inherited,
                      const float *lineage_in, float *lineage_out, void *stream) {
  if (n < 0 || (n > 0 && !chosen) || (inherited && !fitness) || (lineage_out && !lineage_in))
    return fail(PG_ERR_INVALID, "ga_inherit: bad sizes or NULL buffers");
  if (n == 0) return PG_OK;
  hipLaunchKernelGGL(k_inherit, dim3(blocks(n)), dim3(kT), 0, (hipStream_t)stream, chosen, n, fitness, inherited,
                     lineage_in, lineage_out);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

size_t pg_ga_order_workspace_bytes(int32_t n) {
  if (n < 0) return 0;
  const unsigned nn = (unsigned)(n > 0 ? n : 1);
  size_t tb = 0;
  if (rocprim::radix_sort_pairs(nullptr, tb, (const uint32_t *)nullptr, (uint32_t *)nullptr, (const int32_t *)nullptr,
                                (int32_t *)nullptr, nn) != hipSuccess)
    return 0;
  return 2 * align_up((size_t)nn * 4) + align_up((size_t)nn * 4) + align_up(tb > 0 ? tb : 1);
}

int32_t pg_ga_order(int32_t n, int32_t row_lo, const uint8_t *invalid, const float *lineage, int32_t by_length,
                    int32_t *rows, int32_t *count, void *workspace, size_t workspace_bytes, void *stream) {
  if (n < 0 || row_lo < 0 || !count || (n > 0 && !rows))
    return fail(PG_ERR_INVALID, "ga_order: bad sizes or NULL buffers");
  const size_t need = pg_ga_order_workspace_bytes(n);
  if (need == 0 || !workspace || workspace_bytes < need)
    return fail(PG_ERR_INVALID, "ga_order: workspace of %zu bytes needed", need);
  const hipStream_t s = (hipStream_t)stream;
  PG_HIP(hipMemsetAsync(count, 0, sizeof(int32_t), s));
  if (n == 0) return PG_OK;
  char *ws = (char *)workspace;
  uint32_t *keys = (uint32_t *)ws, *keys_out = (uint32_t *)(ws + align_up((size_t)n * 4));
  int32_t *vals = (int32_t *)(ws + 2 * align_up((size_t)n * 4));
  void *temp = ws + 3 * align_up((size_t)n * 4);
  size_t tb = workspace_bytes - 3 * align_up((size_t)n * 4);
  hipLaunchKernelGGL(k_order_keys, dim3(blocks(n)), dim3(kT), 0, s, (int)n, (int)row_lo, invalid, lineage,
                     (int)by_length, keys, vals, count);
  PG_HIP(rocprim::radix_sort_pairs(temp, tb, keys, keys_out, vals, rows, (unsigned)n, 0, 32, s));
  return PG_OK;
}

size_t pg_hof_prepare_cand_workspace_bytes(int32_t hof_n, int32_t k) {
  CandLayout L;
  if (hof_n < 0 || k < 0 || cand_layout(hof_n, k, &L) != PG_OK) return 0;
  return L.total;
}

int32_t pg_hof_prepare_cand(const pg_hof_cand_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  const int hn = a->hof_n, k = a->k;
  if (hn < 0 || k < 0 || (long)hn + k > 0x7fffffffL || (hn > 0 && (!a->hof_fitness || !a->hof_hash)) ||
      (k > 0 && (!a->cand || !a->cand_fitness || !a->rows || !a->cand_hash || !a->packed)) || a->genes < 0 ||
      (k > 0 && a->stride < a->genes) || (a->dtype != PG_F32 && a->dtype != PG_F64))
    return fail(PG_ERR_INVALID, "hof_prepare_cand: bad sizes, dtype or NULL buffers");
  if (k == 0) return PG_OK;
  CandLayout L;
  if (cand_layout(hn, k, &L) != PG_OK) return PG_ERR_HIP;
  if (!a->workspace || a->workspace_bytes < L.total)
    return fail(PG_ERR_INVALID, "hof_prepare_cand: workspace of %zu bytes needed", L.total);
  char *ws = (char *)a->workspace;
  const hipStream_t s = (hipStream_t)stream;
  const int32_t rc = pg_row_hash(a->rows, a->stride, a->cand, k, a->genes, a->dtype, a->cand_hash, stream);
  if (rc != PG_OK) return rc;
  Slot *mt = (Slot *)(ws + L.mt), *ct = (Slot *)(ws + L.ct);
  // both tables and their overflow slots empty: every byte 0xFF
  PG_HIP(hipMemsetAsync(ws + L.mt, 0xFF, L.ct + (size_t)(L.ccap + 1) * sizeof(Slot) - L.mt, s));
  hipLaunchKernelGGL(k_hof_insert, dim3(blocks(hn + k)), dim3(kT), 0, s, a->hof_hash, hn, mt, L.mcap,
                     a->cand_hash, k, ct, L.ccap);
  double *keys = (double *)(ws + L.sort_keys), *sorted = keys + k;
  int32_t *iota = (int32_t *)(ws + L.sort_vals), *order = iota + k;
  hipLaunchKernelGGL(k_cand_keys, dim3(blocks(k)), dim3(kT), 0, s, a->cand_fitness, k, keys, iota);
  size_t tb = L.temp_bytes;
  PG_HIP(rocprim::radix_sort_pairs(ws + L.sort_temp, tb, (const double *)keys, sorted, iota, order, (unsigned)k, 0, 64,
                                   s));
  hipLaunchKernelGGL(k_hof_rank_pack, dim3(blocks(hn + k)), dim3(kT), 0, s, a->hof_fitness,
                     a->hof_hash, hn, a->cand_fitness, a->cand_hash, k,
                     (const double *)sorted, (const int32_t *)order, (const Slot *)mt, L.mcap, (const Slot *)ct,
                     L.ccap, a->packed);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_hof_commit(const pg_hof_commit_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  if (a->m < 0 || a->n_old < 0 || a->genes < 0 || (a->dtype != PG_F32 && a->dtype != PG_F64) ||
      (a->m > 0 && (!a->dst || !a->src || !a->new_hash || !a->fitness_in || !a->new_fitness)) ||
      (a->m > 0 && a->n_old > 0 && ((!a->old_rows && !a->dst_slot) || !a->old_hash)) ||
      (a->m > 0 && (!a->rows || !a->cand || !a->cand_hash)))
    return fail(PG_ERR_INVALID, "hof_commit: bad sizes, dtype or NULL buffers");
  if (a->m == 0) return PG_OK;
  const hipStream_t s = (hipStream_t)stream;
  // (a wave per position; 2048 blocks = 8 per CU cover the largest hall in few passes)
  const dim3 grid((unsigned)std::min<int64_t>(((int64_t)a->m + 3) / 4, 2048));
  if (a->dtype == PG_F64)
    hipLaunchKernelGGL(k_hof_commit<double>, grid, dim3(256), 0, s, (double *)a->dst, a->dst_stride,
                       (const double *)a->old_rows, a->old_stride, (const double *)a->rows, a->rows_stride, a->cand,
                       a->src, (int)a->m, a->n_old, a->genes, a->old_hash, a->cand_hash,
                       a->new_hash, a->fitness_in, a->new_fitness, a->dst_slot);
  else
    hipLaunchKernelGGL(k_hof_commit<float>, grid, dim3(256), 0, s, (float *)a->dst, a->dst_stride,
                       (const float *)a->old_rows, a->old_stride, (const float *)a->rows, a->rows_stride, a->cand,
                       a->src, (int)a->m, a->n_old, a->genes, a->old_hash, a->cand_hash,
                       a->new_hash, a->fitness_in, a->new_fitness, a->dst_slot);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

}  // extern "C"
