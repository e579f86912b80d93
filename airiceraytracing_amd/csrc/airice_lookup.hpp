// airice_lookup.hpp -- the table lookup's per-query code (GetHorizontalDistanceToIntersectionPoint
// _Table and its helpers, MultiRayAirIceRefraction.cc:992-1462), compiled for the device (the
// batch lookup_kernel, airice_lookup.hip) AND the host (the scalar C++ _Table and the
// FindClosest* / GetParValues exports, compat_multiray.cpp): same source, same float->double
// arithmetic, same bits.  Reads the reference makes outside the table are bounded and flagged
// AIRICE_LOOKUP_UNPINNED.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>

#include "airice.h"

namespace airice {

struct LkTable {
  const float* col[AIRICE_TABLE_COLUMNS];  // column c of entry i at col[c][i]
  const float* e;                          // packed copy (airice_lookup_pack) or nullptr
  long long n;
  double stop_h, step_h;  // LoopStopHeight, HeightStepSize of the last table made
  int hsteps, asteps;     // TotalHeightSteps, TotalAngleSteps
  long long rows;         // row records in e (n / asteps), 0: none
  // the packed copy's launch angle of each grid column (column 4 of every table row, which the
  // pack verified), or nullptr: the lookup reads column 4
  const float* ang = nullptr;
};

// Offsets into the packed copy (floats): the pair records, then the row records (128-byte
// aligned), then the angle vector and its verification word (airice.h, AIRICE_LOOKUP_PACK_FLOATS).
__host__ __device__ __forceinline__ long long lk_rows_offset(long long n) {
  return (n * AIRICE_LOOKUP_ENTRY_FLOATS + 31) / 32 * 32;
}
__host__ __device__ __forceinline__ long long lk_angles_offset(long long n, long long asteps) {
  return lk_rows_offset(n) + n / asteps * AIRICE_LOOKUP_ROW_FLOATS;
}
__host__ __device__ __forceinline__ long long lk_angles_ok_offset(long long n, long long asteps) {
  return lk_angles_offset(n, asteps) + (asteps + 3) / 4 * 4;
}
struct LkTxhBins {
  long long s1, e1, s2, e2;
  double c1, c2;
};
struct LkThdBins {
  long long s, e;
  double c;
};

// The 10 interpolated parameters of one table entry (columns 1-10: THD first).
struct LkRec {
  float c[10];
};

__host__ __device__ __forceinline__ LkRec lk_rec(const LkTable& T, long long i, int& fl) {
  LkRec r;
  if (i < 0 || i >= T.n) {
    fl |= AIRICE_LOOKUP_UNPINNED;
#pragma unroll
    for (int c = 0; c < 10; ++c) r.c[c] = __builtin_nanf("");
    return r;
  }
#pragma unroll
  for (int c = 0; c < 10; ++c) r.c[c] = T.col[1 + c][i];
  return r;
}

// Entries i and i + 1 (an interpolation pair) when there is a packed copy and both entries exist
// (false otherwise): columns 2, 3, 5-10 of both from one 64-byte pair record (four 16-byte loads,
// one fabric request), THD (column 1) as the search read it (thd0, thd1: the caller's values of
// entries i, i + 1), the launch angle (column 4) from the angle vector when the pair lies inside
// the row starting at entry abase (else from column 4).
__host__ __device__ __forceinline__ bool lk_pair(const LkTable& T, long long i, float thd0,
                                                 float thd1, long long abase, LkRec& r0,
                                                 LkRec& r1) {
  if (T.e == nullptr || i < 0 || i + 1 >= T.n) return false;
  const float4* p = reinterpret_cast<const float4*>(T.e + (long long)AIRICE_LOOKUP_ENTRY_FLOATS * i);
  const float4 a = p[0], b = p[1], c = p[2], d = p[3];
  const float v[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w,
                       c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
  // record slot k holds parameter par[k] (column 1 + par[k]); lk_pair_fold writes them
  constexpr int par[8] = {1, 2, 4, 5, 6, 7, 8, 9};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    r0.c[par[k]] = v[k];
    r1.c[par[k]] = v[8 + k];
  }
  r0.c[0] = thd0;
  r1.c[0] = thd1;
  const long long j = i - abase;
  if (T.ang != nullptr && abase >= 0 && j >= 0 && j + 1 < T.asteps) {
    r0.c[3] = T.ang[j];
    r1.c[3] = T.ang[j + 1];
  } else {
    r0.c[3] = T.col[4][i];
    r1.c[3] = T.col[4][i + 1];
  }
  return true;
}

// Pair record i (pack time): columns 2, 3, 5-10 of entries i and i + 1 (NaN past the last entry).
__host__ __device__ __forceinline__ void lk_pair_fold(const float* const* col, long long n,
                                                      long long i, float* rec) {
  constexpr int cols[8] = {2, 3, 5, 6, 7, 8, 9, 10};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    rec[k] = col[cols[k]][i];
    rec[8 + k] = i + 1 < n ? col[cols[k]][i + 1] : __builtin_nanf("");
  }
}

__host__ __device__ __forceinline__ double lk_at(const LkTable& T, int c, long long i, int& fl) {
  if (i < 0 || i >= T.n) {
    fl |= AIRICE_LOOKUP_UNPINNED;
    return __builtin_nan("");
  }
  return (double)T.col[c][i];
}

// oneDLinearInterpolation (.cc:992-995)
__host__ __device__ __forceinline__ double lk_interp(double x, double xa, double ya, double xb, double yb) {
  return ya + (yb - ya) * ((x - xa) / (xb - xa));
}

// FindClosestAirTxHeight (.cc:1033-1126): the row of height P and the span of entries with a
// usable THD (not NaN, not in (-inf, 0.01) except exactly 0), scanned inwards from both ends.
__host__ __device__ __forceinline__ long long lk_txh_index(const LkTable& T, double P) {
  const long long step = (long long)floor((P - T.stop_h) / T.step_h);
  return T.hsteps - step - 1;
}

// The span of row `index` (everything of FindClosestAirTxHeight but ClosestVal).
__host__ __device__ __forceinline__ LkTxhBins lk_txh_span(const LkTable& T, long long index, int& fl) {
  const long long max_bin = index * T.asteps + T.asteps - 1;
  const long long min_bin = index * T.asteps;
  double val = -0.001;
  long long start_bin = max_bin;
  bool went = false;
  while ((val != 0 && val < 0.01) || __builtin_isnan(val)) {
    if (start_bin < 0) {  // the reference reads before the table
      fl |= AIRICE_LOOKUP_UNPINNED;
      break;
    }
    val = lk_at(T, 1, start_bin, fl);
    --start_bin;
    went = true;
  }
  if (went) ++start_bin;
  val = -0.001;
  long long end_bin = min_bin;
  went = false;
  while ((val != 0 && val < 0.01) || __builtin_isnan(val)) {
    if (end_bin >= T.n) {  // ... or past its end
      fl |= AIRICE_LOOKUP_UNPINNED;
      break;
    }
    val = lk_at(T, 1, end_bin, fl);
    ++end_bin;
    went = true;
  }
  if (went) --end_bin;
  LkTxhBins b;
  b.s1 = end_bin;
  b.e1 = start_bin;
  b.s2 = b.s1 - T.asteps;
  b.e2 = b.e1 - T.asteps;
  if (b.s2 < 0) b.s2 = b.s1 + T.asteps;
  if (b.e2 < 0) b.e2 = b.e1 + T.asteps;
  b.c1 = 0;
  b.c2 = 0;
  return b;
}

__host__ __device__ __forceinline__ LkTxhBins lk_closest_txh(const LkTable& T, double P, int& fl) {
  const long long index = lk_txh_index(T, P);
  LkTxhBins b = lk_txh_span(T, index, fl);
  b.c1 = fabs(lk_at(T, 0, index, fl) - P);  // sic (.cc:1076): row index used as an entry index
  b.c2 = b.c1;  // ClosestVal2 (.cc:1123) is the same expression
  return b;
}

// Row record (packed copy, after the entry records): the span of row `index` and the table values
// the lookup reads at its ends, folded by airice_lookup_pack from the same code as above.  Used
// only for rows whose scans stay inside the table (ok), so the flags are unchanged.
//
// FindClosestTHD's first four bisection steps on a span (s, e) depend on the query only through
// the comparisons: from a given span the midpoints form a fixed binary tree of depth 4 (15 nodes,
// breadth-first: node k's successors 2k + 1 after s = mid, 2k + 2 after e = mid).  The record holds
// the THD value at each node for the row's own span (s1, e1) and for the span the second
// interpolation height searches (s2, e2): a query then takes its first four steps from two 128-byte
// lines it reads anyway instead of four dependent gathers into the THD column, and the rest of
// the search and the linear scan from one short window of that column (lk_closest_thd_tree).
// threads per block of the batch lookup_kernel (round 5, 1e6 random queries incl. the fallback
// pass, same outputs: 64 100.3-100.9, 128 100.6-100.9, 256 101.5-102.3, 512 104.0-104.6 us)
constexpr int kLkBlock = 128;      // (its LDS window
                                   // has one column per thread: lk_closest_thd_tree)
constexpr int kLkTreeNodes = 15;  // bisection steps 0-3
constexpr int kLkWindow = 12;     // THD entries the steps 4-7 and the scan may read
struct LkTree {
  float v[kLkTreeNodes];
};
struct LkRow {
  LkTxhBins b;
  double c1v;      // column 0 at entry `index` (ClosestVal's operand)
  double h1, h2;   // column 0 at s1, at s2 (s2 < n - 1)
  double mt1, mt2; // column 1 (THD) at s1, at s2
  bool tree1, tree2;  // the node values below are usable (every node's midpoint inside the table)
  const float* rec;   // the row record: tree 1 at floats 8-22, tree 2 at floats 32-46
  float4 top1, top2;    // nodes 0-3 of each tree (levels 0 and 1 without a dependent read)
  float4 top1b, top2b;  // nodes 4-7 (level 2 with node 3)
};
__host__ __device__ __forceinline__ float lk_bits_f(int32_t i) {
  float f;
  std::memcpy(&f, &i, sizeof(f));
  return f;
}
__host__ __device__ __forceinline__ int32_t lk_bits_i(float f) {
  int32_t i;
  std::memcpy(&i, &f, sizeof(i));
  return i;
}
// THD values at the 15 nodes of the bisection tree of span (s, e) (pack time).  False when a
// node's midpoint lies outside the table (the lane then searches the column: lk_closest_thd).
__host__ __device__ __forceinline__ bool lk_tree_fold(const LkTable& T, long long s, long long e,
                                                      float* out) {
  long long ss[kLkTreeNodes], ee[kLkTreeNodes];
  bool live[kLkTreeNodes];
  ss[0] = s;
  ee[0] = e;
  live[0] = true;
  bool ok = true;
  for (int k = 0; k < kLkTreeNodes; ++k) {
    out[k] = 0.0f;
    const bool inner = 2 * k + 2 < kLkTreeNodes;
    bool split = live[k] && ee[k] - ss[k] >= 3;
    long long mid = 0;
    if (split) {
      mid = (ss[k] + ee[k]) / 2;  // FindClosestTHD's midpoint (.cc:1142)
      if (mid < 0 || mid >= T.n) {
        ok = false;
        split = false;
      } else {
        out[k] = T.col[1][mid];
      }
    }
    if (inner) {
      live[2 * k + 1] = live[2 * k + 2] = split;
      ss[2 * k + 1] = mid;  // v - P > 0: StartIndex = mid
      ee[2 * k + 1] = ee[k];
      ss[2 * k + 2] = ss[k];  // v - P < 0: EndIndex = mid
      ee[2 * k + 2] = mid;
    }
  }
  return ok;
}

// The search span of the second interpolation height, from the first's (.cc:1118-1121).
__host__ __device__ __forceinline__ void lk_span2(const LkTable& T, LkTxhBins& b) {
  b.s2 = b.s1 - T.asteps;
  b.e2 = b.e1 - T.asteps;
  if (b.s2 < 0) b.s2 = b.s1 + T.asteps;
  if (b.e2 < 0) b.e2 = b.e1 + T.asteps;
}

// Fold row r (pack time), AIRICE_LOOKUP_ROW_FLOATS floats in two 128-byte lines:
//   line 0: {s1, e1 (int bits), col0[r], col0[s1], col0[s2], col1[s1], col1[s2], ok (int bits)},
//           the tree of (s1, e1) (floats 8-22), tree bits (float 23: 1 = tree 1, 2 = tree 2);
//   line 1: the tree of (s2, e2) (floats 32-46).
__host__ __device__ __forceinline__ void lk_row_fold(const LkTable& T, long long r, float* rec) {
  int fl = 0;
  const LkTxhBins b = lk_txh_span(T, r, fl);
  const bool s2_used = b.s2 < T.n - 1;
  const bool ok = fl == 0 && b.s1 >= 0 && b.s1 < T.n && r < T.n && b.s1 < (1LL << 31) &&
                  b.e1 >= -(1LL << 31) && b.e1 < (1LL << 31) && b.s2 >= 0;
  for (int k = 0; k < AIRICE_LOOKUP_ROW_FLOATS; ++k) rec[k] = 0.0f;
  rec[0] = lk_bits_f((int32_t)(ok ? b.s1 : 0));
  rec[1] = lk_bits_f((int32_t)(ok ? b.e1 : 0));
  rec[2] = ok ? T.col[0][r] : 0.0f;
  rec[3] = ok ? T.col[0][b.s1] : 0.0f;
  rec[4] = ok && s2_used ? T.col[0][b.s2] : 0.0f;
  rec[5] = ok ? T.col[1][b.s1] : 0.0f;
  rec[6] = ok && s2_used ? T.col[1][b.s2] : 0.0f;
  rec[7] = lk_bits_f(ok ? 1 : 0);
  int trees = 0;
  if (ok) {
    LkTxhBins b2 = b;  // the span lk_row rebuilds from (s1, e1)
    lk_span2(T, b2);
    if (lk_tree_fold(T, b2.s1, b2.e1, rec + 8)) trees |= 1;
    if (lk_tree_fold(T, b2.s2, b2.e2, rec + 32)) trees |= 2;
  }
  rec[23] = lk_bits_f(trees);
}
__host__ __device__ __forceinline__ const float4* lk_row_rec(const LkTable& T, long long index) {
  return reinterpret_cast<const float4*>(T.e + lk_rows_offset(T.n) +
                                         index * AIRICE_LOOKUP_ROW_FLOATS);
}
__host__ __device__ __forceinline__ void lk_tree_unpack(const float4* p, LkTree& T_) {
  float* t = T_.v;
  // floats 0-14 of the 4 float4 at p
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 a = p[q];
    t[4 * q] = a.x;
    t[4 * q + 1] = a.y;
    t[4 * q + 2] = a.z;
    if (4 * q + 3 < kLkTreeNodes) t[4 * q + 3] = a.w;
  }
}
__host__ __device__ __forceinline__ bool lk_row(const LkTable& T, long long index, LkRow& R) {
  if (T.e == nullptr || index < 0 || index >= T.rows) return false;
  const float4* p = lk_row_rec(T, index);
  const float4 a = p[0], c = p[1];
  if (lk_bits_i(c.w) == 0) return false;
  R.b.s1 = lk_bits_i(a.x);
  R.b.e1 = lk_bits_i(a.y);
  lk_span2(T, R.b);
  R.c1v = a.z;
  R.h1 = a.w;
  R.h2 = c.x;
  R.mt1 = c.y;
  R.mt2 = c.z;
  R.rec = reinterpret_cast<const float*>(p);
  R.top1 = p[2];
  R.top2 = p[8];
  R.top1b = p[3];
  R.top2b = p[9];
  const int trees = lk_bits_i(R.rec[23]);
  R.tree1 = (trees & 1) != 0;
  R.tree2 = (trees & 2) != 0;
  return true;
}

// FindClosestTHD (.cc:1128-1169).  With a packed table the final pair's record carries the
// parameters lk_row_params interpolates (have_pair).  abase: first entry of the searched row (the
// angle vector's origin), or -1.
struct LkThdPair {
  LkRec r1, r2;  // entries index1, index2
  bool have_pair = false;
};
__host__ __device__ __forceinline__ LkThdBins lk_closest_thd(const LkTable& T, double P, long long s, long long e,
                                            int& fl, LkThdPair& pr, long long abase = -1) {
#pragma unroll 1
  for (int i = 0; i < 8; ++i) {
    if (e - s >= 3) {
      const long long mid = (s + e) / 2;
      const double v = lk_at(T, 1, mid, fl);
      if (v - P > 0) s = mid;
      if (v - P < 0) e = mid;
    }
  }
  double minimum = 100000000000.0;
  long long index2 = 0;
#pragma unroll 1
  for (long long ip = s; ip < e + 1; ++ip) {
    const double v = lk_at(T, 1, ip, fl);
    const double minval = fabs(v - P);
    if (minval < minimum && v > P) {
      minimum = minval;
    } else {
      index2 = ip;
      break;
    }
  }
  const long long index1 = index2 - 1;
  const double v2 = lk_at(T, 1, index2, fl);
  const double v1 = lk_at(T, 1, index1, fl);
  pr.have_pair = lk_pair(T, index1, (float)v1, (float)v2, abase, pr.r1, pr.r2);
  minimum = fabs(P - v2);
  if (minimum > fabs(P - v1)) minimum = fabs(P - v1);
  return LkThdBins{index1, index2, minimum};
}

// v[j] of N values by a binary multiplexer on the bits of j (0 <= j < N): selects only, so the
// values stay in registers (an equality chain is turned back into an indexed private array).
template <int N>
__host__ __device__ __forceinline__ float lk_mux(const float* v, int j) {
  float m[N];
#pragma unroll
  for (int i = 0; i < N; ++i) m[i] = v[i];
#pragma unroll
  for (int w = 1; w < N; w *= 2) {
    const bool hi = (j & w) != 0;
#pragma unroll
    for (int i = 0; i + w < N; i += 2 * w) m[i] = hi ? m[i + w] : m[i];
  }
  return m[0];
}

// One step of lk_closest_thd's bisection (.cc:1140-1147) on indices s <= e below 2^31 and the
// THD value v at their midpoint: s = mid if v - P > 0, e = mid if v - P < 0, and otherwise (equal,
// NaN) `fin`, since every later step would repeat this one unchanged.  Returns the branch taken.
__host__ __device__ __forceinline__ bool lk_step32(double v, double P, int& s, int& e, bool& fin) {
  const int mid = (int)(((unsigned)s + (unsigned)e) >> 1);  // (s + e) / 2, s, e >= 0
  const bool up = v - P > 0, down = v - P < 0;
  s = up ? mid : s;
  e = down ? mid : e;
  fin = fin || !(up || down);
  return up;
}

// lk_closest_thd from a row record's tree (the first four steps) and kLkWindow consecutive THD
// values (the rest of the steps and the scan): the same index1, index2, minimum and pair, read
// from the packed copy.  False -- the caller then runs lk_closest_thd -- when the span left after
// the tree is wider than the window, the search ends on a span of more than 3 entries (an equal
// or NaN midpoint), the scan runs off its end without a break, or the pair has no packed record;
// every value it reads lies inside the table, so no flag changes.  Indices are 32-bit here (the
// row fold admits spans below 2^31 only).
// win: on the device, this lane's column of the caller's LDS window (lookup_kernel: kLkWindow rows
// of kLkBlock lanes, row stride kLkBlock; without one the lane takes the column path); on the
// host the window is a private array.
__host__ __device__ __forceinline__ bool lk_closest_thd_tree(const LkTable& T, double P, long long s_in,
                                                             long long e_in, const float* t,
                                                             float4 top, float4 topb,
                                                             LkThdBins& out, LkThdPair& pr,
                                                             long long abase, float* win) {
  if (s_in < 0 || e_in < s_in || T.n < kLkWindow || T.n >= (1LL << 31)) return false;
  int s = (int)s_in, e = (int)e_in;
  bool fin = false;
  int k = 0;  // tree node of the current step
#pragma unroll
  for (int lvl = 0; lvl < 4; ++lvl) {
    fin = fin || e - s < 3;
    if (!fin) {
      // the node's value: levels 0-2 from the record's first 32 bytes, read with the row, level 3
      // from the record (one dependent 4-byte read of a line the lane has read)
      const float v = lvl == 0   ? top.x
                      : lvl == 1 ? (k == 1 ? top.y : top.z)
                      : lvl == 2 ? (k == 3 ? top.w : k == 4 ? topb.x : k == 5 ? topb.y : topb.z)
                                 : t[k];
      const bool up = lk_step32((double)v, P, s, e, fin);
      k = 2 * k + (up ? 1 : 2);
    }
  }
  if (e - s >= kLkWindow) return false;
  const int n32 = (int)T.n;
  const int base = s <= n32 - kLkWindow ? s : n32 - kLkWindow;  // the window covers [s, e]
  // the window, indexed per lane: in lookup_kernel in the block's LDS (one column of 4-byte slots
  // per lane, kLkWindow rows kLkBlock lanes apart: conflict-free, and each read one instruction
  // where a register multiplexer takes 11 selects; the lane reads only what it wrote), otherwise
  // a private array
  const float* src = T.col[1] + base;
#if defined(__HIP_DEVICE_COMPILE__)
  // device callers pass their window (a private array indexed per lane would live in scratch)
  if (win == nullptr) return false;
  float* w = win;
  constexpr int ws = kLkBlock;
#else
  float priv[kLkWindow];
  float* w = priv;
  constexpr int ws = 1;
  (void)win;
#endif
  // three 16-byte loads at 4-byte alignment (gfx950 vector memory takes unaligned dwordx4)
  typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
#pragma unroll
  for (int q = 0; q < kLkWindow / 4; ++q) {
    const f4u a = reinterpret_cast<const f4u*>(src)[q];
    w[(4 * q) * ws] = a.x;
    w[(4 * q + 1) * ws] = a.y;
    w[(4 * q + 2) * ws] = a.z;
    w[(4 * q + 3) * ws] = a.w;
  }
#pragma unroll
  for (int i = 4; i < 8; ++i) {
    fin = fin || e - s < 3;
    if (!fin) {
      const int mid = (int)(((unsigned)s + (unsigned)e) >> 1);
      lk_step32((double)w[(mid - base) * ws], P, s, e, fin);
    }
  }
  if (e - s > 2) return false;
  // the linear scan (.cc:1150-1160) over the <= 3 entries of [s, e]
  const int j0 = s - base;  // j0 + 2 <= 11 when the third entry exists (e <= base + 11)
  const int j1 = j0 + 1 < kLkWindow ? j0 + 1 : kLkWindow - 1;
  const int j2 = j0 + 2 < kLkWindow ? j0 + 2 : kLkWindow - 1;
  const float sv[3] = {w[j0 * ws], w[j1 * ws], w[j2 * ws]};
  double minimum = 100000000000.0;
  int index2 = 0;
  bool brk = false;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (!brk && s + j <= e) {
      const double v = (double)sv[j];
      const double minval = fabs(v - P);
      if (minval < minimum && v > P) {
        minimum = minval;
      } else {
        index2 = s + j;
        brk = true;
      }
    }
  }
  if (!brk) return false;
  const long long index1 = (long long)index2 - 1;
  // THD at the pair from the window (index2 is in [s, e]; index1 too unless index2 == base)
  const float t2 = w[(index2 - base) * ws];
  const float t1 = index2 > base ? w[(index2 - 1 - base) * ws] : (index1 >= 0 ? T.col[1][index1] : 0.0f);
  if (!lk_pair(T, index1, t1, t2, abase, pr.r1, pr.r2)) return false;
  pr.have_pair = true;
  const double v2 = (double)t2, v1 = (double)t1;
  minimum = fabs(P - v2);
  if (minimum > fabs(P - v1)) minimum = fabs(P - v1);
  out = LkThdBins{index1, (long long)index2, minimum};
  return true;
}

// The 10 parameters of one table row at horizontal distance D (.cc:1199-1240 / 1250-1289).
// tree: the row record's bisection tree of (s, e) when use_tree.
// abase: first entry of the row the span lies in (the angle vector's origin), or -1.
__host__ __device__ __forceinline__ void lk_row_params(const LkTable& T, double D, long long s, long long e,
                                              double par[10], double* closest, int& fl,
                                              const double* max_thd_row = nullptr,
                                              const float* tree = nullptr,
                                              float4 tree_top = float4{},
                                              float4 tree_topb = float4{},
                                              long long abase = -1, float* win = nullptr) {
  const double max_thd = max_thd_row != nullptr ? *max_thd_row : lk_at(T, 1, s, fl);
  if (D <= max_thd) {
    LkThdPair pr;
    LkThdBins b;
    if (tree == nullptr ||
        !lk_closest_thd_tree(T, D, s, e, tree, tree_top, tree_topb, b, pr, abase, win)) {
      pr.have_pair = false;
      b = lk_closest_thd(T, D, s, e, fl, pr, abase);
    }
    *closest = b.c;
    if (b.c != 0) {
      // b.e == b.s + 1 (index1 = index2 - 1)
      const LkRec rs = pr.have_pair ? pr.r1 : lk_rec(T, b.s, fl);
      const LkRec re = pr.have_pair ? pr.r2 : lk_rec(T, b.e, fl);
      const double x1 = pr.have_pair ? (double)pr.r1.c[0] : lk_at(T, 1, b.s, fl);
      const double x2 = pr.have_pair ? (double)pr.r2.c[0] : lk_at(T, 1, b.e, fl);
#pragma unroll
      for (int ip = 0; ip < 10; ++ip)
        par[ip] = lk_interp(D, x1, (double)rs.c[ip], x2, (double)re.c[ip]);
    } else {
      const LkRec r = pr.have_pair ? pr.r2 : lk_rec(T, b.s + 1, fl);
#pragma unroll
      for (int ip = 0; ip < 10; ++ip) par[ip] = (double)r.c[ip];
    }
  } else {
#pragma unroll
    for (int ip = 0; ip < 10; ++ip) par[ip] = -1e9;
  }
}

// GetParValues (.cc:1172-1302) for a Tx height inside the table's range (win: lk_closest_thd_tree)
__host__ __device__ __forceinline__ void lk_par_values(const LkTable& T, double H, double D, double* h1,
                                       double par1[10], double* h2, double par2[10], int& fl,
                                       float* win = nullptr) {
  const double min_h = lk_at(T, 0, T.n - 1, fl);
  LkRow R;  // packed row record: the span and its end values without the scans
  const long long index = lk_txh_index(T, H);
  const bool fast = lk_row(T, index, R);
  LkTxhBins b;
  if (fast) {
    b = R.b;
    b.c1 = fabs(R.c1v - H);
    b.c2 = b.c1;
  } else {
    b = lk_closest_txh(T, H, fl);
  }
  double c1 = 0;
  *h1 = fast ? R.h1 : lk_at(T, 0, b.s1, fl);
  // the rows of the two spans: the height's own, and the one s2 moved to (.cc:1118-1121)
  const long long abase1 = index * T.asteps;
  const long long abase2 = b.s2 < b.s1 ? abase1 - T.asteps : abase1 + T.asteps;
  lk_row_params(T, D, b.s1, b.e1, par1, &c1, fl, fast ? &R.mt1 : nullptr,
                fast && R.tree1 ? R.rec + 8 : nullptr, R.top1, R.top1b, abase1, win);
  *h2 = *h1;
  if (b.c1 != 0 && H > min_h && b.s2 < T.n - 1) {
    *h2 = fast ? R.h2 : lk_at(T, 0, b.s2, fl);
    double c2 = 0;
    lk_row_params(T, D, b.s2, b.e2, par2, &c2, fl, fast ? &R.mt2 : nullptr,
                  fast && R.tree2 ? R.rec + 32 : nullptr, R.top2, R.top2b, abase2, win);
  } else {
#pragma unroll
    for (int ip = 0; ip < 10; ++ip) par2[ip] = par1[ip];
  }
}

// GetHorizontalDistanceToIntersectionPoint_Table (.cc:1305-1462) for one query (metres): out9
// in the reference's argument order, *good = CheckSolution.  Returns true when the query hits the
// one-sided extrapolation case, whose outputs the minimizer fallback (.cc:1418-1420) rewrites.
__host__ __device__ __forceinline__ bool lk_query(const LkTable& T, double H, double D, double d2r, double out[9],
                                  bool* good_out, int& fl, float* win = nullptr) {
  const double max_h = lk_at(T, 0, 0, fl);
  const double min_h = lk_at(T, 0, T.n - 1, fl);
  double x1 = 0, x2 = 0, y1 = 0, y2 = 0;
  double piv[10];
  unsigned set = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) piv[i] = 0;
  if (H <= max_h && H >= min_h && H > 0) {
    double par1[10], par2[10];
    lk_par_values(T, H, D, &x1, par1, &x2, par2, fl, win);
    // interpolation in height (.cc:1376-1401); a parameter missing at both heights ends the
    // loop writing its value into slot 9 (the reference sets ipar = 9 before the store)
    bool done = false;
#pragma unroll
    for (int ip = 0; ip < 10; ++ip) {
      if (!done) {
        y1 = par1[ip];
        y2 = par2[ip];
        double v = 0;
        const bool missing = (y1 == -1e9 || y2 == -1e9);
        if (x1 != x2 && !missing) {
          v = lk_interp(H, x1, y1, x2, y2);
        } else if (x1 == x2 && y1 == y2) {
          v = par1[ip];
        }
        if ((x1 == x2 || missing) && y2 == -1e9 && y1 == -1e9) {
          piv[9] = v;
          set |= 1u << 9;
          done = true;
        } else {
          piv[ip] = v;
          set |= 1u << ip;
        }
      }
    }
  }
  if (set != 0x3ffu) fl |= AIRICE_LOOKUP_UNPINNED;
  const double thd = piv[0];
  const bool one_sided = (y1 == -1e9 && y2 != -1e9) || (y2 == -1e9 && y1 != -1e9);
  bool good = true;
  if (y2 == -1e9 && y1 == -1e9) good = false;
  if (H > max_h) good = false;
  if (H < min_h) good = false;
  if (H < 0) good = false;
  if ((fabs(thd - D) / D > 0.01 && D <= 100) || (fabs(thd - D) > 1 && D > 100)) good = false;
  *good_out = good;
  if (one_sided) {
    // finished by the fallback pass: every output slot is rewritten there, and the checks
    // above are completed with CheckSolBool and launchAngle < 0
    fl |= AIRICE_LOOKUP_FALLBACK;
    return true;
  }
  const double la = piv[3] * d2r;  // pi/180 (.cc:1410)
  if (la < 0) good = false;
  *good_out = good;
  out[0] = good ? piv[1] * 100 : 0.0;  // opticalPathLengthInIce
  out[1] = good ? piv[2] * 100 : 0.0;  // opticalPathLengthInAir
  out[2] = piv[8] * 100;               // geometricalPathLengthInIce
  out[3] = piv[7] * 100;               // geometricalPathLengthInAir
  out[4] = good ? la : 0.0;            // launchAngle
  out[5] = good ? piv[4] * 100 : 0.0;  // horizontalDistanceToIntersectionPoint
  out[6] = piv[5];                     // transmissionCoefficientS
  out[7] = piv[6];                     // transmissionCoefficientP
  out[8] = piv[9] * d2r;               // RecievedAngleInIce
  return false;
}

// The lookup's view of a table (host: the launchers build it per call).
inline LkTable lk_table(const airice_lookup_table* t) {
  LkTable T;
  for (int c = 0; c < AIRICE_TABLE_COLUMNS; ++c) T.col[c] = t->table + (size_t)c * t->ld;
  T.e = t->entries;
  T.n = (long long)t->n_entries;
  T.stop_h = t->loop_stop_height;
  T.step_h = t->height_step;
  T.hsteps = t->total_height_steps;
  T.asteps = t->total_angle_steps;
  T.rows = T.e != nullptr ? T.n / T.asteps : 0;
  // the angle vector; lookup_kernel drops it when the pack found a row with other angles
  T.ang = T.e != nullptr ? T.e + lk_angles_offset(T.n, T.asteps) : nullptr;
  return T;
}

}  // namespace airice
