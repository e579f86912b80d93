// airice_lookup.hip -- batched GetHorizontalDistanceToIntersectionPoint_Table on gfx950.
//
//  lookup_kernel : one lane per (Tx height, horizontal distance, Rx depth) query against one
//                  antenna's HBM-resident table (11 float columns, SoA).  The lane runs the
//                  reference's bin search and two-level linear interpolation:
//                    FindClosestAirTxHeight (.cc:1033-1126)  row of the Tx height and the
//                                                            valid-THD span of that row,
//                    FindClosestTHD         (.cc:1128-1169)  8 bisection steps + linear scan,
//                    GetParValues           (.cc:1172-1302)  10 columns at 2 heights
//                                                            (one 128-byte packed record per
//                                                            interpolation pair when packed),
//                    _Table                 (.cc:1305-1462)  interpolation in height, checks.
//                  Lanes that hit the one-sided extrapolation case (.cc:1418) are flagged and
//                  finished by the masked minimizer pass (launch_lookup_fallback,
//                  airice_kernels.hip), which reproduces the reference's fallback call.
//
// Cost model: every lane gathers its own lines, so the kernel is bound by the 128-byte lines it
// pulls from L2 / the Infinity Cache per query, not by bytes.  With the packed copy a query reads
// the row record (two lines: the span, its end values and the THD values of the first four
// bisection steps of both heights), then per height one short window of the THD column (steps 4-7
// and the scan, 48 B) and one pair record (128 B): ~7 lines, against ~13 when the bisection
// gathered each midpoint from the THD column.
// Reads the reference makes outside the table (a row with no valid THD, index -1 in
// FindClosestTHD) are bounded here and reported as AIRICE_LOOKUP_UNPINNED.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "airice.h"
#include "airice_internal.h"
#include "airice_lookup.hpp"

namespace airice {

namespace {

static_assert(kLkBlock % 64 == 0, "the pack kernels' grids (airice_lookup.hpp)");

__global__ __launch_bounds__(kLkBlock) void lookup_angles_kernel(LkTable T, float* __restrict__ e) {
  const long long j = (long long)blockIdx.x * kLkBlock + threadIdx.x;
  float* ang = e + lk_angles_offset(T.n, T.asteps);
  if (j < T.asteps) ang[j] = j < T.n ? T.col[4][j] : __builtin_nanf("");
  if (j == 0) *reinterpret_cast<int*>(e + lk_angles_ok_offset(T.n, T.asteps)) = 1;
}

// Then one lane per pair record (lk_pair_fold: entries i and i + 1); the column reads are coalesced
// across the wave and each wave writes one contiguous 4 KB run of records.  Each lane also checks
// its entry's launch angle against the first row's (bit for bit): the table's column 4 is the
// angle grid in every row (.cc:2084-2105), and a table where it is not keeps the column path.
__global__ __launch_bounds__(kLkBlock) void lookup_pack_kernel(LkTable T, float* __restrict__ e) {
  const long long i = (long long)blockIdx.x * kLkBlock + threadIdx.x;
  if (i >= T.n) return;
  float c[AIRICE_LOOKUP_ENTRY_FLOATS];
  lk_pair_fold(T.col, T.n, i, c);
  float4* p = reinterpret_cast<float4*>(e + (long long)AIRICE_LOOKUP_ENTRY_FLOATS * i);
#pragma unroll
  for (int q = 0; q < AIRICE_LOOKUP_ENTRY_FLOATS / 4; ++q)
    p[q] = make_float4(c[4 * q], c[4 * q + 1], c[4 * q + 2], c[4 * q + 3]);
  if (lk_bits_i(T.col[4][i]) != lk_bits_i(T.col[4][i % T.asteps]))
    atomicAnd(reinterpret_cast<int*>(e + lk_angles_ok_offset(T.n, T.asteps)), 0);
}

// Row records after the entry records: one lane per full table row (lk_row_fold).
__global__ __launch_bounds__(kLkBlock) void lookup_rows_kernel(LkTable T, float* __restrict__ e) {
  const long long r = (long long)blockIdx.x * kLkBlock + threadIdx.x;
  if (r >= T.rows) return;
  float rec[AIRICE_LOOKUP_ROW_FLOATS];
  lk_row_fold(T, r, rec);
  float4* p = reinterpret_cast<float4*>(e + lk_rows_offset(T.n) + r * AIRICE_LOOKUP_ROW_FLOATS);
#pragma unroll
  for (int q = 0; q < AIRICE_LOOKUP_ROW_FLOATS / 4; ++q)
    p[q] = make_float4(rec[4 * q], rec[4 * q + 1], rec[4 * q + 2], rec[4 * q + 3]);
}


}  // namespace

int launch_lookup_pack(const airice_lookup_table* t, float* e, hipStream_t st) {
  const long long n = (long long)t->n_entries;
  if (n == 0) return AIRICE_OK;
  LkTable T = lk_table(t);
  T.e = e;
  T.rows = n / T.asteps;
  hipLaunchKernelGGL(lookup_angles_kernel, dim3((unsigned)((T.asteps + kLkBlock - 1) / kLkBlock)),
                     dim3(kLkBlock), 0, st, T, e);
  hipLaunchKernelGGL(lookup_pack_kernel, dim3((unsigned)((n + kLkBlock - 1) / kLkBlock)),
                     dim3(kLkBlock), 0, st, T, e);
  if (T.rows > 0)
    hipLaunchKernelGGL(lookup_rows_kernel, dim3((unsigned)((T.rows + kLkBlock - 1) / kLkBlock)),
                       dim3(kLkBlock), 0, st, T, e);
  return hipGetLastError() == hipSuccess ? AIRICE_OK : AIRICE_EHIP;
}

}  // namespace airice
