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
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

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

struct Above {  // the full hall's admission filter: fitness strictly above its worst
  const double *fitness;
  double worst;
  __device__ bool operator()(int32_t i) const { return fitness[i] > worst; }
};

__global__ void k_hof_iota(int32_t *out, int n) {
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i < n) out[i] = i;
}

__global__ void k_hof_cand_gather(const int32_t *cand32, int k, const double *fitness, int64_t *cand,
                                  double *cand_fitness) {
  const int j = blockIdx.x * kThreads + threadIdx.x;
  if (j >= k) return;
  const int i = cand32[j];
  cand[j] = i;
  cand_fitness[j] = fitness[i];
}

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

int32_t rank_classes_core(int hn, const double *hof_fitness, const uint64_t *hof_hash, int k,
                          const double *cand_fitness, const uint64_t *cand_hash, int64_t *packed, char *ws,
                          const Layout &L, hipStream_t s) {
  const int n = hn + k;
  double *fkeys = (double *)(ws + L.keys_a), *fsorted = (double *)(ws + L.keys_b);
  uint64_t *hkeys = (uint64_t *)(ws + L.keys_a), *hsorted = (uint64_t *)(ws + L.keys_b);
  int32_t *iota = (int32_t *)(ws + L.iota), *order = (int32_t *)(ws + L.order);
  int32_t *rank = (int32_t *)(ws + L.rank), *flag = (int32_t *)(ws + L.flag), *cls = (int32_t *)(ws + L.cls);
  void *temp = ws + L.temp;
  size_t temp_bytes = L.temp_bytes;
  const unsigned g = blocks_for(n);
  // ranks: radix sort is stable, so equal fitness keeps age order
  hipLaunchKernelGGL(k_hof_age_keys, dim3(g), dim3(kThreads), 0, s, hof_fitness, hn, cand_fitness, k, fkeys, iota);
  PG_HIP(rocprim::radix_sort_pairs(temp, temp_bytes, fkeys, fsorted, iota, order, (unsigned)n, 0, 64, s));
  hipLaunchKernelGGL(k_hof_rank, dim3(g), dim3(kThreads), 0, s, order, hn, n, rank);
  // classes: sort the hashes, count the distinct values in sorted order
  hipLaunchKernelGGL(k_hof_hash_keys, dim3(g), dim3(kThreads), 0, s, hof_hash, hn, cand_hash, k, hkeys, iota);
  temp_bytes = L.temp_bytes;
  PG_HIP(rocprim::radix_sort_pairs(temp, temp_bytes, hkeys, hsorted, iota, order, (unsigned)n, 0, 64, s));
  hipLaunchKernelGGL(k_hof_new_class, dim3(g), dim3(kThreads), 0, s, hsorted, n, flag);
  temp_bytes = L.temp_bytes;
  PG_HIP(rocprim::inclusive_scan(temp, temp_bytes, flag, cls, (size_t)n, rocprim::plus<int32_t>(), s));
  hipLaunchKernelGGL(k_hof_pack, dim3(blocks_for(n > k ? n : k)), dim3(kThreads), 0, s, rank, order, cls, n,
                     cand_fitness, k, packed);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

// pg_hof_prepare's workspace: the rank/class layout for hof_n + pop_n entries,
// then the candidate list, their fitness, the device count and select's storage.
struct PrepLayout {
  Layout rc;
  size_t cand32, cfit, count, sel, total, sel_bytes;
};

int32_t prep_layout_for(int hn, int pn, const double *fitness, PrepLayout *P) {
  if (layout_for(hn + pn, &P->rc) != PG_OK) return PG_ERR_HIP;
  size_t sel = 0;
  if (rocprim::select(nullptr, sel, rocprim::counting_iterator<int32_t>(0), (int32_t *)nullptr, (int32_t *)nullptr,
                      (size_t)(pn > 0 ? pn : 1), Above{fitness, 0.0}) != hipSuccess)
    return fail(PG_ERR_HIP, "hof_prepare: rocPRIM select storage query failed");
  size_t off = P->rc.total;
  auto take = [&](size_t bytes) {
    const size_t at = off;
    off += align_up(bytes);
    return at;
  };
  const size_t pp = (size_t)(pn > 0 ? pn : 1);
  P->cand32 = take(pp * 4);
  P->cfit = take(pp * 8);
  P->count = take(8);
  P->sel_bytes = sel > 0 ? sel : 1;
  P->sel = take(P->sel_bytes);
  P->total = off;
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
  return rank_classes_core(hn, a->hof_fitness, a->hof_hash, k, a->cand_fitness, a->cand_hash, a->packed,
                           (char *)a->workspace, L, (hipStream_t)stream);
}

size_t pg_hof_prepare_workspace_bytes(int32_t hof_n, int32_t pop_n) {
  PrepLayout P;
  if (hof_n < 0 || pop_n < 0 || prep_layout_for(hof_n, pop_n, nullptr, &P) != PG_OK) return 0;
  return P.total;
}

int32_t pg_hof_prepare(const pg_hof_prepare_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  const int hn = a->hof_n, pn = a->pop_n;
  if (hn < 0 || pn < 0 || (long)hn + pn > 0x7fffffffL || !a->k || (hn > 0 && (!a->hof_fitness || !a->hof_hash)) ||
      (pn > 0 && (!a->fitness || !a->rows || !a->cand || !a->hashes || !a->packed)) || a->genes < 0 ||
      (pn > 0 && a->stride < a->genes) || (a->dtype != PG_F32 && a->dtype != PG_F64))
    return fail(PG_ERR_INVALID, "hof_prepare: bad sizes, dtype or NULL buffers");
  *a->k = 0;
  if (pn == 0) return PG_OK;
  PrepLayout P;
  if (prep_layout_for(hn, pn, a->fitness, &P) != PG_OK) return PG_ERR_HIP;
  if (!a->workspace || a->workspace_bytes < P.total)
    return fail(PG_ERR_INVALID, "hof_prepare: workspace of %zu bytes needed", P.total);
  char *ws = (char *)a->workspace;
  int32_t *cand32 = (int32_t *)(ws + P.cand32), *count = (int32_t *)(ws + P.count);
  double *cfit = (double *)(ws + P.cfit);
  const hipStream_t s = (hipStream_t)stream;
  int k = pn;
  if (a->filter) {
    size_t sel_bytes = P.sel_bytes;
    PG_HIP(rocprim::select(ws + P.sel, sel_bytes, rocprim::counting_iterator<int32_t>(0), cand32, count, (size_t)pn,
                           Above{a->fitness, a->worst}, s));
    int32_t k_host = 0;
    PG_HIP(hipMemcpyAsync(&k_host, count, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    PG_HIP(hipStreamSynchronize(s));  // the one sync: the scan's input size
    k = k_host;
  } else {
    hipLaunchKernelGGL(k_hof_iota, dim3(blocks_for(pn)), dim3(kThreads), 0, s, cand32, pn);
  }
  *a->k = k;
  if (k == 0) return PG_OK;
  if (hn > 0) PG_HIP(hipMemcpyAsync(a->hashes, a->hof_hash, (size_t)hn * 8, hipMemcpyDeviceToDevice, s));
  const int32_t rc = pg_row_hash(a->rows, a->stride, cand32, k, a->genes, a->dtype, a->hashes + hn, stream);
  if (rc != PG_OK) return rc;
  hipLaunchKernelGGL(k_hof_cand_gather, dim3(blocks_for(k)), dim3(kThreads), 0, s, cand32, k, a->fitness, a->cand,
                     cfit);
  Layout L;
  if (layout_for(hn + k, &L) != PG_OK) return PG_ERR_HIP;
  if (L.total > P.rc.total) return fail(PG_ERR_INVALID, "hof_prepare: rank/class layout grew with fewer entries");
  return rank_classes_core(hn, a->hof_fitness, a->hashes, k, cfit, a->hashes + hn, a->packed, ws, L, s);
}

}  // extern "C"
