// pg_hof.hip -- the device half of HallOfFame.update (DEAP, eaSimple's
// halloffame.update(offspring), main.py:165-170): for the old members and the
// candidate rows together, each entry's rank in ascending (fitness, age)
// order and a dense similarity class of the row hashes, packed for the host
// scan (pg_hof_update) in one buffer.  One C-ABI call replaces a dozen
// tensor ops (and torch.unique's host sync): two rocPRIM radix sorts, one
// scan and four small kernels on the caller's stream.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "pg_eval.hpp"

namespace pg {
namespace {

constexpr int kThreads = 256;

inline unsigned blocks_for(int n) { return (unsigned)((n + kThreads - 1) / kThreads); }

// by-age keys: the members reversed (items order is descending (fitness, age),
// so the oldest member, entry hof_n - 1, has age 0), then the candidates.
__global__ void k_hof_age_keys(const double *hof_fitness, int hof_n, const double *cand_fitness, int k,
                               double *keys, int32_t *iota) {
  const int i = blockIdx.x * kThreads + threadIdx.x;
  const int n = hof_n + k;
  if (i >= n) return;
  keys[i] = i < hof_n ? hof_fitness[hof_n - 1 - i] : cand_fitness[i - hof_n];
  iota[i] = i;
}

// rank of entry e (items order for members, then candidates) from the sorted
// age positions: sorted slot s holds age position p.
__global__ void k_hof_rank(const int32_t *order, int hof_n, int n, int32_t *rank) {
  const int s = blockIdx.x * kThreads + threadIdx.x;
  if (s >= n) return;
  const int p = order[s];
  rank[p < hof_n ? hof_n - 1 - p : p] = s;
}

__global__ void k_hof_hash_keys(const uint64_t *hof_hash, int hof_n, const uint64_t *cand_hash, int k,
                                uint64_t *keys, int32_t *iota) {
  const int i = blockIdx.x * kThreads + threadIdx.x;
  const int n = hof_n + k;
  if (i >= n) return;
  keys[i] = i < hof_n ? hof_hash[i] : cand_hash[i - hof_n];
  iota[i] = i;
}

__global__ void k_hof_new_class(const uint64_t *sorted, int n, int32_t *flag) {
  const int s = blockIdx.x * kThreads + threadIdx.x;
  if (s >= n) return;
  flag[s] = (s > 0 && sorted[s] != sorted[s - 1]) ? 1 : 0;
}

// packed[e] = rank[e] | class[e] << 32 (class = inclusive count of new hashes
// up to e's sorted slot); packed[n + j] = candidate j's fitness bits.
__global__ void k_hof_pack(const int32_t *rank, const int32_t *hash_order, const int32_t *cls_sorted, int n,
                           const double *cand_fitness, int k, int64_t *packed) {
  const int s = blockIdx.x * kThreads + threadIdx.x;
  if (s < n) {
    const int e = hash_order[s];
    packed[e] = (int64_t)(uint32_t)rank[e] | ((int64_t)cls_sorted[s] << 32);
  }
  if (s < k) packed[n + s] = __double_as_longlong(cand_fitness[s]);
}

// rank[e] must be written before k_hof_pack reads it at a permuted index, so
// the pack runs as its own launch after k_hof_rank (stream order).

struct Layout {
  size_t keys_a, keys_b, iota, order, rank, flag, cls, temp, total;
  size_t temp_bytes;
};

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

int32_t layout_for(int n, Layout *L) {
  size_t t_sort_f64 = 0, t_sort_u64 = 0, t_scan = 0;
  if (rocprim::radix_sort_pairs(nullptr, t_sort_f64, (const double *)nullptr, (double *)nullptr,
                                (const int32_t *)nullptr, (int32_t *)nullptr, (unsigned)n) != hipSuccess ||
      rocprim::radix_sort_pairs(nullptr, t_sort_u64, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                (const int32_t *)nullptr, (int32_t *)nullptr, (unsigned)n) != hipSuccess ||
      rocprim::inclusive_scan(nullptr, t_scan, (const int32_t *)nullptr, (int32_t *)nullptr, (size_t)n,
                              rocprim::plus<int32_t>()) != hipSuccess)
    return fail(PG_ERR_HIP, "hof_rank_classes: rocPRIM temporary-storage query failed");
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t at = off;
    off += align_up(bytes);
    return at;
  };
  const size_t nn = (size_t)(n > 0 ? n : 1);
  L->keys_a = take(nn * 8);
  L->keys_b = take(nn * 8);
  L->iota = take(nn * 4);
  L->order = take(nn * 4);
  L->rank = take(nn * 4);
  L->flag = take(nn * 4);
  L->cls = take(nn * 4);
  L->temp_bytes = std::max(std::max(t_sort_f64, t_sort_u64), std::max(t_scan, (size_t)1));
  L->temp = take(L->temp_bytes);
  L->total = off;
  return PG_OK;
}

}  // namespace
}  // namespace pg

using namespace pg;

extern "C" {

size_t pg_hof_rank_classes_workspace_bytes(int32_t n) {
  Layout L;
  if (n < 0 || layout_for(n, &L) != PG_OK) return 0;
  return L.total;
}

int32_t pg_hof_rank_classes(const pg_hof_rank_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  const int hn = a->hof_n, k = a->k;
  if (hn < 0 || k < 0 || (long)hn + k > 0x7fffffffL || !a->packed ||
      (hn > 0 && (!a->hof_fitness || !a->hof_hash)) || (k > 0 && (!a->cand_fitness || !a->cand_hash)))
    return fail(PG_ERR_INVALID, "hof_rank_classes: bad sizes or NULL buffers");
  const int n = hn + k;
  if (n == 0) return PG_OK;
  Layout L;
  if (layout_for(n, &L) != PG_OK) return PG_ERR_HIP;
  if (!a->workspace || a->workspace_bytes < L.total)
    return fail(PG_ERR_INVALID, "hof_rank_classes: workspace of %zu bytes needed", L.total);
  char *ws = (char *)a->workspace;
  double *fkeys = (double *)(ws + L.keys_a), *fsorted = (double *)(ws + L.keys_b);
  uint64_t *hkeys = (uint64_t *)(ws + L.keys_a), *hsorted = (uint64_t *)(ws + L.keys_b);
  int32_t *iota = (int32_t *)(ws + L.iota), *order = (int32_t *)(ws + L.order);
  int32_t *rank = (int32_t *)(ws + L.rank), *flag = (int32_t *)(ws + L.flag), *cls = (int32_t *)(ws + L.cls);
  void *temp = ws + L.temp;
  size_t temp_bytes = L.temp_bytes;
  const hipStream_t s = (hipStream_t)stream;
  const unsigned g = blocks_for(n);
  // ranks: radix sort is stable, so equal fitness keeps age order
  hipLaunchKernelGGL(k_hof_age_keys, dim3(g), dim3(kThreads), 0, s, a->hof_fitness, hn, a->cand_fitness, k, fkeys,
                     iota);
  PG_HIP(rocprim::radix_sort_pairs(temp, temp_bytes, fkeys, fsorted, iota, order, (unsigned)n, 0, 64, s));
  hipLaunchKernelGGL(k_hof_rank, dim3(g), dim3(kThreads), 0, s, order, hn, n, rank);
  // classes: sort the hashes, count the distinct values in sorted order
  hipLaunchKernelGGL(k_hof_hash_keys, dim3(g), dim3(kThreads), 0, s, a->hof_hash, hn, a->cand_hash, k, hkeys, iota);
  temp_bytes = L.temp_bytes;
  PG_HIP(rocprim::radix_sort_pairs(temp, temp_bytes, hkeys, hsorted, iota, order, (unsigned)n, 0, 64, s));
  hipLaunchKernelGGL(k_hof_new_class, dim3(g), dim3(kThreads), 0, s, hsorted, n, flag);
  temp_bytes = L.temp_bytes;
  PG_HIP(rocprim::inclusive_scan(temp, temp_bytes, flag, cls, (size_t)n, rocprim::plus<int32_t>(), s));
  hipLaunchKernelGGL(k_hof_pack, dim3(blocks_for(n > k ? n : k)), dim3(kThreads), 0, s, rank, order, cls, n,
                     a->cand_fitness, k, a->packed);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

}  // extern "C"
