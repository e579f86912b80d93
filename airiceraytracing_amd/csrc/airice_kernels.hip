// airice_kernels.hip -- gfx950 kernels + stream-ordered launchers of libairice.so.
//
//  table_kernel   : one lane per (TxHeight, launch angle) ray of MakeRayTracingTable
//                   (MultiRayAirIceRefraction.cc:2079-2122 loop body -> GetRayTracingSolutions
//                   .cc:1796-2017), writes the 11 float table columns (.cc:2101-2111) and,
//                   optionally, the 18 doubles of dummy[] for parity checks.
//  rays_kernel    : the same ray for arbitrary (angle, height) lists.
//  solve_kernel   : one lane per query of Air2IceRayTracing (.cc:1464-1616): bracket set-up,
//                   the 0.05-degree probe loop, GSL-bisection emulation (tolerance 1e-9,
//                   40 iterations) over a THD-only evaluator, one full evaluation at the root.
//                   VARIANT selects MultiRay (dummy[17]) / pythonwrapper (dummy[15]) outputs.
//  hdtip_kernel   : GetHorizontalDistanceToIntersectionPoint (.cc:945-989), cm in/out.
//  trace_kernel   : pythonwrapper TraceIceToAir (TraceIceToAir.C:5-73) rows of 10.
//
// Data layout in HBM: structure-of-arrays, column c of item i at out[c*ld + i], so each
// wave's store of one column is one contiguous 256 B (f32) / 512 B (f64) segment.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "airice.h"
#include "airice_lookup.hpp"
#include "airice_device.hpp"
#include "airice_internal.h"
#include "airice_lean.hpp"

namespace airice {

constexpr double kSpeedC = 299792458.0;  // .h:30
constexpr int kBlock = 256;
#ifndef AIRICE_OUT_WAVES
#define AIRICE_OUT_WAVES 1
#endif
constexpr int kOutWaves = AIRICE_OUT_WAVES;  // stage-2 kernels: minimum waves per SIMD (1: no cap)
// trace_out_kernel held to 8 waves/SIMD: 64 VGPRs without scratch (94 uncapped, 5 waves), cfg5
// 1e7 trace calls 2.059-2.064 against 2.074-2.100 ms, same outputs (profiles/r06_ab/stage2_waves_ab.log);
// solve_out / hdtip_out capped at 5-8 waves measured within noise or slower (8: spills), uncapped
#ifndef AIRICE_TRACE_OUT_WAVES
#define AIRICE_TRACE_OUT_WAVES 8
#endif
constexpr int kTraceOutWaves = AIRICE_TRACE_OUT_WAVES;
// Table launch shape: 256-thread blocks at 8 waves/SIMD (64 VGPRs), measured best of 64 / 128 /
// 256 / 512 threads, 7 / 8 waves and 1 / 2 rays per lane.
#ifndef AIRICE_TABLE_BLOCK
#define AIRICE_TABLE_BLOCK 256
#endif
constexpr int kTableBlock = AIRICE_TABLE_BLOCK;  // (A/B builds: -DAIRICE_TABLE_BLOCK=...)
constexpr int kTableWaves = 8;
// debug builds: shader-clock stamps of the one-query kernels (tools/scalar_stamps.py,
// tools/ray_stamps.py) and the minimizer's evaluation counts by sorted position (tools/wave_evals.py)
#ifndef AIRICE_SCALAR_STAMP
#define AIRICE_SCALAR_STAMP 0
#endif
#ifndef AIRICE_RAY_STAMP
#define AIRICE_RAY_STAMP 0
#endif
#ifndef AIRICE_NO_CHECK
#define AIRICE_NO_CHECK 0
#endif
#ifndef AIRICE_SORTED_STATS
#define AIRICE_SORTED_STATS 0
#endif
// debug build: roots_kernel writes shader-clock stamps instead of evaluation counts
// (AIRICE_SOLVE_STATS, 4 ints per query: entry, sorted, inputs at hand, solved; tools/roots_stamps.py)
#ifndef AIRICE_ROOTS_STAMP
#define AIRICE_ROOTS_STAMP 0
#endif
constexpr int kStatsInts = AIRICE_ROOTS_STAMP == 3 ? 8 : AIRICE_ROOTS_STAMP == 2 ? 7 : AIRICE_ROOTS_STAMP ? 4 : 3;
// evaluation-free bisection steps of the root finder per loop trip (as compare-and-select)
constexpr int kLeanUnroll = 4;
// table stores take an SGPR column base and a 32-bit lane byte offset (global_store saddr form):
// launches are split at 2^30 rays so that 4 k < 2^32
constexpr long long kMaxLaunchRays = 1LL << 30;
// table launches of fewer rays store their columns at agent scope (table_ray's SC1)
constexpr long long kAgentStoreRays = 1LL << 24;

// ---------------------------------------------------------------------------
// Forward ray: GetRayTracingSolutions (.cc:1796-2017).  d[] = dummy[0..17].
// The layer loop follows the reference (each layer re-derives L from the incidence angle
// it receives, .cc:1871) with the running sine of identity (2).
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ Endpoint stop_of(const DevMedium& M, int l) {
  Endpoint r = M.stop[0];
  r = pick(l == 1, M.stop[1], r);
  r = pick(l == 2, M.stop[2], r);
  r = pick(l == 3, M.stop[3], r);
  return r;
}

// Fresnel T_S, T_P (.cc:285-337) at the incidence whose sine is v (identity (2):
// sin(asin(v) r2d d2r) = v, cos = sqrt(1 - v^2) on [0, 90] degrees).
// ratio = n1 / n2 (folded on the host, IceConsts::n_ratio).  The two quotients have positive
// denominators (n1, n2 > 0 and ct, sqterm >= 0, never both 0): div_pos.
__host__ __device__ __forceinline__ void fresnel_from_sine(double n1, double n2, double ratio, double v,
                                                  double& tS, double& tP) {
  const double st = v, ct = fast_sqrt(1 - v * v);
  const double a = ratio * st;
  const double sqterm = fast_sqrt(1 - a * a);
  double num = n1 * ct - n2 * sqterm;
  double den = n1 * ct + n2 * sqterm;
  tS = 1 + div_pos(num, den);
  if (__builtin_isnan(tS)) tS = 0;
  num = n1 * sqterm - n2 * ct;
  den = n1 * sqterm + n2 * ct;
  tP = (1 - div_pos(num, den)) * ratio;
  if (__builtin_isnan(tP)) tP = 0;
}

// Stop end of the Tx layer `top`.  Rays of one wave almost always share their Tx layer (a
// wave covers <= 2 table rows), so the entry is read with a wave-uniform (scalar) index;
// a wave that straddles a layer boundary falls back to per-lane selects.
__host__ __device__ __forceinline__ TopEnd topend_of(const IceConsts& I, int top) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int tu = __builtin_amdgcn_readfirstlane(top);
  if (__ballot(top != tu) == 0) return I.topend[tu];
#endif
  TopEnd r = I.topend[0];
#pragma unroll
  for (int l = 1; l < kMaxLayers; ++l) {
    const bool c = (top == l);
    const TopEnd& e = I.topend[l];
    r = TopEnd{c ? e.x : r.x,       c ? e.n : r.n,       c ? e.y2 : r.y2, c ? e.Ay : r.Ay,
               c ? e.invC : r.invC, c ? e.invCc : r.invCc, c ? e.Cx : r.Cx, c ? e.ACx : r.ACx};
  }
  return r;
}

// Everything of a ray that depends on its Tx height only: the Tx layer and the Tx layer's
// segment folded like the lower layers' (Tx endpoint -> the layer's stop end, or the ice).  The
// table computes it once per row into LDS (a block spans few rows); other launches per lane.
struct RowConst {
  SegConst seg;  // Tx endpoint -> stop end of the Tx layer (zero-length case resolved)
  double H;
  int top;       // MaxLayers - SkipLayersAbove - 1
  int any;       // top >= bot: at least one air layer
};

__host__ __device__ __forceinline__ RowConst row_const(const DevMedium& M, const IceConsts& I, double H) {
  RowConst rc;
  rc.H = H;
  rc.top = top_layer(M, H);
  rc.any = rc.top >= I.bot;
  const Endpoint T = air_endpoint(M, H);
  const TopEnd R_ = topend_of(I, rc.top);
  // zero-length (Tx exactly on the layer's lower bound / the ice): reuse the Tx end
  const bool zl = (R_.x == T.x);
  SegConst& s = rc.seg;
  s.Tn = T.n;
  s.Ty2 = T.y2;
  s.TAy = T.Ay;
  s.Rn = zl ? T.n : R_.n;
  s.Ry2 = zl ? T.y2 : R_.y2;
  s.RAy = zl ? T.Ay : R_.Ay;
  s.ratio = T.n / s.Rn;
  s.invC = zl ? T.invC : R_.invC;
  s.invCc = zl ? T.invC * (1.0 / kSpeedC) : R_.invCc;
  s.dCx = zl ? 0.0 : R_.Cx - T.Cx;
  s.dACx = zl ? 0.0 : R_.ACx - T.ACx;
  return rc;
}

// sin(x) for the start angle's radians, x = (180 - theta) pi/180 in [0, pi/2] for every launch
// angle in [90, 180]: odd Taylor polynomial to x^23 (truncation < 2^-59 relative on the range);
// other arguments go to ocml's sin.
__host__ __device__ __forceinline__ double sin_start(double x) {
  if (!(x >= 0.0 && x <= 1.5707963267948966)) return sin(x);
  const double x2 = x * x;
  // (-1)^k / (2k+1)!, k = 11 .. 1, as doubles
  double p = __builtin_fma(x2, -0x1.761b41316381ap-75, kc(0x1.71b8ef6dcf572p-66));  // 1/23!, 1/21!
  p = __builtin_fma(x2, p, kc(-0x1.2f49b46814157p-57));                             // 1/19!
  p = __builtin_fma(x2, p, kc(0x1.952c77030ad4ap-49));                              // 1/17!
  p = __builtin_fma(x2, p, kc(-0x1.ae7f3e733b81fp-41));                             // 1/15!
  p = __builtin_fma(x2, p, kc(0x1.6124613a86d09p-33));                              // 1/13!
  p = __builtin_fma(x2, p, kc(-0x1.ae64567f544e4p-26));                             // 1/11!
  p = __builtin_fma(x2, p, kc(0x1.71de3a556c734p-19));                              // 1/9!
  p = __builtin_fma(x2, p, kc(-0x1.a01a01a01a01ap-13));                             // 1/7!
  p = __builtin_fma(x2, p, kc(0x1.1111111111111p-7));                               // 1/5!
  p = __builtin_fma(x2, p, kc(-0x1.5555555555555p-3));                              // 1/3!
  return __builtin_fma(x * x2, p, x);
}

// I.lower[il].ratio for a lane-varying il (selects)
__host__ __device__ __forceinline__ double sel_lower_ratio(const IceConsts& I, int il) {
  double r = I.lower[0].ratio;
#pragma unroll
  for (int l = 1; l < kMaxLayers; ++l) r = (il == l) ? I.lower[l].ratio : r;
  return r;
}

// want_inc: dummy[12] (the incidence angle on the ice, one asin) is not a table column
// (.cc:2101-2111), so table launches without the double output skip it.
// top_hi >= 0: a wave-uniform upper bound of the lanes' Tx layers (the table block's first row);
// the lower layers then run as one loop over a uniform layer index, their SegConst read with
// scalar loads one layer at a time, instead of one inlined copy per layer.  Same operations in
// the same order either way.
// A1: the launch's A_air is exactly 1 (MultiRayAirIceRefraction.h:99, the table's medium), so
// the products with it are dropped (exact: x * 1.0 == x).
template <bool A1 = false>
__host__ __device__ __forceinline__ void ray_solution_row(const DevMedium& M, const IceConsts& I,
                                                 const RowConst& rc, double theta, bool in_ice,
                                                 double* d, bool want_inc,
                                                 const double* tab = &kLogTable[0][0],
                                                 int top_hi = -1,
                                                 const double* v_start = nullptr) {
  const double H = rc.H;
  const int top = rc.top;
  const int bot = I.bot;
  const double Aair = A1 ? 1.0 : M.A_air;
  const double A2 = Aair * Aair;
  // sine of StartAngle (.cc:1863); v_start: the same value, formed by the caller
  double v = v_start != nullptr ? *v_start : sin_start((180 - theta) * M.d2r);
  double thd_air = 0.0, t_air = 0.0, geo_air = 0.0;
  const bool any = rc.any != 0;
  if (any) {
    // n_layer1 == Getnz_air(StartHeight) == nzTx: Snell into a layer is the identity
    const Segment s = segment_const(rc.seg, Aair, A2, sin_asin(v), true, v, tab);
    thd_air += s.thd;
    t_air += s.t;
    geo_air += s.geo;
  }
  // lower layers: both ends folded on the host (I.lower, scalar reads)
  if (top_hi >= 0) {
#pragma clang loop unroll(disable)
    for (int il = top_hi - 1; il >= bot; --il) {
      if (il < top) {
        // v is a segment's output sine here (already sin_asin'd: sin_asin is idempotent)
        const Segment s = segment_const(I.lower[il], Aair, A2, v, true, v, tab);
        thd_air += s.thd;
        t_air += s.t;
        geo_air += s.geo;
      }
    }
  } else {
#pragma unroll
    for (int il = kMaxLayers - 2; il >= 0; --il) {
      if (il >= top || il < bot) continue;
      const Segment s = segment_const(I.lower[il], Aair, A2, v, true, v, tab);
      thd_air += s.thd;
      t_air += s.t;
      geo_air += s.geo;
    }
  }
  // IncidentAngleonIce = last layer's receive angle; 0 when no air layer (.cc:1832, 1881)
  double inc = 0.0;
  if (want_inc) inc = any ? k_asin(v) * M.r2d : 0.0;
  const double vinc = any ? v : 0.0;
  double thd_ice = 0.0, t_ice = 0.0, geo_ice = 0.0, recv_ice = 0.0;
  if (in_ice) {
    // .cc:1897-1922: n_layer1 = Getnz_air(IceLayerHeight), Rx = -AntennaDepth, Tx = 0
    const double A2i = M.A_ice * M.A_ice;
    const double u = sin_asin(I.n_ratio * vinc);
    double v2;
    const Segment s = segment_const(I.iceseg, M.A_ice, A2i, u, false, v2, tab);
    thd_ice += s.thd;
    t_ice += s.t;
    geo_ice += s.geo;
    recv_ice = k_asin(v2) * M.r2d;
  }
  double tS, tP;
  fresnel_from_sine(I.n_air_ice, I.n_ice0, I.n_ratio, vinc, tS, tP);
  d[0] = 0;
  d[1] = H;
  d[2] = thd_air + thd_ice;
  d[3] = thd_air;
  d[4] = thd_ice;
  d[5] = (t_ice + t_air) * kSpeedC;
  d[6] = t_air * kSpeedC;
  d[7] = t_ice * kSpeedC;
  d[8] = (t_ice + t_air) * 1e9;
  d[9] = t_air * 1e9;
  d[10] = t_ice * 1e9;
  d[11] = theta;
  d[12] = inc;
  d[13] = recv_ice;
  d[14] = tS;
  d[15] = tP;
  d[16] = geo_air;
  d[17] = geo_ice;
}

// Per-lane form (rays, minimizer evaluations): the row constants of its own Tx height.
__host__ __device__ __forceinline__ void ray_solution(const DevMedium& M, const IceConsts& I, double theta,
                                             double H, bool in_ice, double* d,
                                             bool want_inc = true) {
  const RowConst rc = row_const(M, I, H);
  ray_solution_row(M, I, rc, theta, in_ice, d, want_inc);
}

struct TableArgs {
  double start_h, stop_h, step_h;
  double start_a, stop_a, step_a;
  double inv_asteps;  // 1.0 / asteps (row of ray k without an integer division)
  int hsteps, asteps;
  int row0, in_ice;
  int n;              // rays of this launch (< 2^31; launch_table splits larger grids)
  int rows_per_block; // LDS rows a block's set of rays may span
  int half;           // rays per set (R = 2: ceil(n / 2); R = 1: n)
  size_t ld;
  const struct RowConst* rc;  // the grid's row constants (all hsteps rows, computed once per
                              // medium and grid: row_consts_cached), or nullptr
  const double* vs;           // sin of the start angle of every column (angle_sines_cached), or
                              // nullptr
};

// Debug timeline (AIRICE_TABLE_TRACE=<file>, tools/wave_timeline.py): per wave, the 100 MHz
// s_memrealtime at entry and exit plus HW_ID / XCC_ID.  Not part of the API.
struct WaveTrace {
  unsigned long long t0, t1;
  unsigned long long c0, c1;  // s_memtime (shader clock) at entry and exit: the in-kernel clock
  unsigned hw_id, xcc_id;
};

// Tx height of grid row ihei (.cc:2080, 2089-2091; separate mul and add, no contraction).
__device__ __forceinline__ double row_height(const TableArgs& G, int ihei) {
  double H = G.start_h - G.step_h * ihei;
  if (H != G.stop_h && ihei == G.hsteps - 1) H = G.stop_h;
  return H;
}

// Row (within the launch) of ray k: the double quotient k / asteps is within 1 of the integer
// one for k < 2^31, then fixed up.
__device__ __forceinline__ int ray_row(const TableArgs& G, int k) {
  int r = (int)((double)k * G.inv_asteps);
  if (r * G.asteps > k) --r;
  if ((r + 1) * G.asteps <= k) ++r;
  return r;
}

// One table entry: ray k of the launch (row r, row-major over TxH rows x launch angles).
// Launch angle of column iang of the grid (.cc:2085, 2092-2094).
__device__ __forceinline__ double table_angle(const TableArgs& G, int iang) {
  double th = G.start_a + G.step_a * iang;
  if (iang == G.asteps - 1) th = G.stop_a;
  return th;
}

template <bool A1, bool SC1>
__device__ __forceinline__ void table_ray(const DevMedium& M, const IceConsts& I,
                                          const TableArgs& G, const RowConst& rc, int r, int k,
                                          float* __restrict__ table, double* __restrict__ full,
                                          const double* tab, int top_hi) {
  const int iang = k - r * G.asteps;
  const double th = table_angle(G, iang);
  double d[18];
  // the start-angle sine of every grid column, formed once per angle grid (angle_sines_kernel);
  // launches captured into a graph before their grid was cached form it here
  double vs;
  if (G.vs != nullptr)
    vs = G.vs[iang];
  else
    vs = sin_start((180 - th) * M.d2r);
  ray_solution_row<A1>(M, I, rc, th, G.in_ice != 0, d, full != nullptr, tab, top_hi, &vs);
  const size_t ld = G.ld;
  // AllTableAllAntData columns (.cc:2101-2111): the column base is wave-uniform, the lane's byte
  // offset fits 32 bits (k < 2^30 per launch)
  {
    char* tb = reinterpret_cast<char*>(table);
    const size_t ldb = ld * sizeof(float);
    const uint32_t off = (uint32_t)k * 4u;
    // (non-temporal stores: cfg2 28.9 -> 29.9 us, same bits)
    // SC1: the column stores at agent scope (global_store ... sc1), for launches short enough that
    // the lines they leave dirty in the XCDs' L2s are a visible part of the launch: cfg2 28.9-29.2
    // -> 27.8-28.2 us, the same table (without any table store the kernel takes 25.6 us); at cfg4
    // size plain stores are faster (20.8 against 21.9 ms per build)
    auto st = [&](int c, double v) {
      float* p = reinterpret_cast<float*>(tb + c * ldb + off);
      if constexpr (SC1)
        st_agent(p, (float)v);
      else
        *p = (float)v;
    };
    st(0, d[1]);
    st(1, d[2]);
    st(2, d[7]);
    st(3, d[6]);
    st(4, d[11]);
    st(5, d[3]);
    st(6, d[14]);
    st(7, d[15]);
    st(8, d[16]);
    st(9, d[17]);
    st(10, d[13]);
  }
  if (full != nullptr) {
#pragma unroll
    for (int c = 0; c < 18; ++c) full[c * ld + k] = d[c];
  }
}

// Table launch: one ray per lane, ray k = block * 256 + threadIdx.x (each wave's column store one
// contiguous 256 B segment).  The block first stages the Tx-height-only constants of the (few) rows
// it spans into LDS -- copied from the grid's row-constant cache, or, when the launch has none, one
// lane per row computes them, so the exp / layer scans / top-layer folding run once per row
// instead of once per wave -- then every lane traces its ray.
// (Measured and rejected, DESIGN.md §5: persistent grid-stride and atomic-chunk schedules -- the
// loop around the inlined ray body raises register pressure to 160 VGPRs, or 330 B/lane of scratch
// when capped at 64, and runs 2.7x / 7x slower -- and two rays per lane.)
// The work of one table block (kTableBlock rays of one antenna's grid), shared by the single- and
// the multi-antenna kernels.
template <bool TRACE, bool A1, bool SC1>
__device__ __forceinline__ void table_block(const DevMedium& M, const IceConsts& I,
                                            const TableArgs& G, float* __restrict__ table,
                                            double* __restrict__ full,
                                            WaveTrace* __restrict__ trace, unsigned block) {
  constexpr int BS = kTableBlock;
  extern __shared__ __align__(16) unsigned char smem[];
  RowConst* rows = reinterpret_cast<RowConst*>(smem);
  // the log table (16 B x 2^kLogTableBits) staged in LDS: 16-byte entries, (1 << kLogTableBits) / BS per thread
  __shared__ __align__(16) double s_logtab[1 << kLogTableBits][2];
#pragma unroll
  for (unsigned t = threadIdx.x; t < (1u << kLogTableBits); t += BS) {
    s_logtab[t][0] = kLogTable[t][0];
    s_logtab[t][1] = kLogTable[t][1];
  }
  const unsigned wave = block * (BS / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (TRACE && lane == 0) {
    trace[wave].t0 = __builtin_amdgcn_s_memrealtime();
    trace[wave].c0 = __builtin_amdgcn_s_memtime();
  }
  const int k0 = (int)block * BS;
  const int ke = min(k0 + BS, G.n);  // end of this block's rays
  const int r0 = k0 < ke ? ray_row(G, k0) : 0;
  {
    const int nrows = k0 < ke ? ray_row(G, ke - 1) - r0 + 1 : 0;
    for (int t = threadIdx.x; t < nrows; t += BS)
      rows[t] = G.rc != nullptr ? G.rc[G.row0 + r0 + t]
                                : row_const(M, I, row_height(G, G.row0 + r0 + t));
  }
  __syncthreads();
  const int k = k0 + (int)threadIdx.x;
  if (k0 < G.n) {  // block-uniform
    // the block's first row has the highest Tx, so its Tx layer bounds every lane's (top_layer is
    // monotone in the height)
    const int top_hi = __builtin_amdgcn_readfirstlane(rows[0].top);
    __builtin_assume(top_hi >= 0);
    if (k < G.n) {
      const int r = ray_row(G, k);
      table_ray<A1, SC1>(M, I, G, rows[r - r0], r, k, table, full, &s_logtab[0][0], top_hi);
    }
  }
  if (TRACE && lane == 0) {
    trace[wave].t1 = __builtin_amdgcn_s_memrealtime();
    trace[wave].c1 = __builtin_amdgcn_s_memtime();
    trace[wave].hw_id = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
    trace[wave].xcc_id = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
  }
}

// waves_per_eu(8): 64 VGPRs at 8 waves/SIMD, measured on par or slightly ahead of 67 VGPRs at 7.
template <bool TRACE, bool A1, bool SC1>
__global__ __launch_bounds__(kTableBlock) __attribute__((amdgpu_waves_per_eu(kTableWaves, kTableWaves))) void table_kernel(
                                                   DevMedium M, IceConsts I, TableArgs G,
                                                   float* __restrict__ table,
                                                   double* __restrict__ full,
                                                   WaveTrace* __restrict__ trace) {
  table_block<TRACE, A1, SC1>(M, I, G, table, full, trace, blockIdx.x);
}

// Several antennas' tables in one grid (airice_table_launch_multi): the blocks of antenna a are
// [begin[a], begin[a+1]); its per-antenna constants (IceConsts, TableArgs: antenna depth, stop
// height) come from global memory, read with scalar loads since the index is block-uniform.
// One launch ramp and one drain for all antennas instead of one per table.
constexpr int kMaxAntennas = 32;
struct MultiMap {
  int n_ant;
  int begin[kMaxAntennas + 1];
  float* table[kMaxAntennas];
};

template <bool A1, bool SC1>
__global__ __launch_bounds__(kTableBlock) __attribute__((amdgpu_waves_per_eu(kTableWaves, kTableWaves))) void table_multi_kernel(
    DevMedium M, const IceConsts* __restrict__ Iv, const TableArgs* __restrict__ Gv, MultiMap map) {
  int a = 0;
  for (int j = 1; j < map.n_ant; ++j) a += (int)blockIdx.x >= map.begin[j];
  a = __builtin_amdgcn_readfirstlane(a);
  table_block<false, A1, SC1>(M, Iv[a], Gv[a], map.table[a], nullptr, nullptr,
                         blockIdx.x - (unsigned)map.begin[a]);
}

// Row constants of a whole grid (row_consts_cached): one row per lane, the table block's own
// row_const on the same heights, so the cached values are the bits the block would compute.
__global__ __launch_bounds__(256) void rowconst_kernel(DevMedium M, IceConsts I, TableArgs G,
                                                       RowConst* __restrict__ out) {
  const int r = (int)(blockIdx.x * 256 + threadIdx.x);
  if (r < G.hsteps) out[r] = row_const(M, I, row_height(G, r));
}

// Start-angle sines of a grid's columns (angle_sines_cached): the table ray's own expression.
__global__ __launch_bounds__(256) void angle_sines_kernel(DevMedium M, TableArgs G,
                                                          double* __restrict__ out) {
  const int a = (int)(blockIdx.x * 256 + threadIdx.x);
  if (a < G.asteps) out[a] = sin_start((180 - table_angle(G, a)) * M.d2r);
}

// One forward ray spread over a wave (the one-query GetRayTracingSolutions call): the running
// sine chain is cheap, so every lane walks it and knows the input sine of each segment; lane 0
// then traces the Tx-layer segment, lanes 1-3 the lower layers (top-1, top-2, top-3 while >= bot),
// lane 4 the segment in the ice, all at once, while the angle outputs and the Fresnel
// coefficients (functions of the chain's sines only) run beside them on every lane; the sums are
// formed in ray_solution_row's order from the lanes' values.  The same operations on the same
// values as ray_solution (hence the same bits), with the ~1,000-deep one-lane chain cut to about
// one segment.
__device__ __forceinline__ void ray_solution_wave(const DevMedium& M, const IceConsts& I,
                                                  double theta, double H, bool in_ice, double* d,
                                                  const double* tab,
                                                  unsigned long long* ts = nullptr) {
  const int lane = (int)(threadIdx.x & 63);
  const RowConst rc = row_const(M, I, H);
#if AIRICE_RAY_STAMP
  ts[1] = __builtin_amdgcn_s_memtime() + (unsigned long long)(0.0 * rc.seg.ratio);
#endif
  const int top = rc.top, bot = I.bot;
  const bool any = rc.any != 0;
  const double A2 = M.A_air * M.A_air, A2i = M.A_ice * M.A_ice;
  // the chain: input sine of every segment, and the sine after the air layers
  double v = sin_start((180 - theta) * M.d2r);
  double sin_in[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  bool on[5] = {false, false, false, false, false};
  if (any) {
    sin_in[0] = sin_asin(v);
    on[0] = true;
    v = sin_asin(rc.seg.ratio * sin_in[0]);
  }
#pragma unroll
  for (int j = 1; j <= 3; ++j) {
    const int il = top - j;
    if (il >= bot && il >= 0) {
      sin_in[j] = v;
      on[j] = true;
      v = sin_asin(sel_lower_ratio(I, il) * v);
    }
  }
  const double vinc = any ? v : 0.0;
  const double u_ice = sin_asin(I.n_ratio * vinc);
  sin_in[4] = u_ice;
  on[4] = in_ice;
#if AIRICE_RAY_STAMP
  ts[2] = __builtin_amdgcn_s_memtime() + (unsigned long long)(0.0 * u_ice);
#endif
  // this lane's segment
  const int j = lane < 5 ? lane : 0;
  SegConst S = rc.seg;
  double sj = sin_in[0];
#pragma unroll
  for (int q = 1; q <= 4; ++q) {
    const bool me = j == q;
    sj = me ? sin_in[q] : sj;
  }
  const int il = top - j;
#pragma unroll
  for (int l = 0; l < kMaxLayers; ++l) {
    const bool me = j >= 1 && j <= 3 && il == l;
    const SegConst& c = I.lower[l];
    S = SegConst{me ? c.Tn : S.Tn,       me ? c.Ty2 : S.Ty2,     me ? c.TAy : S.TAy,
                 me ? c.Rn : S.Rn,       me ? c.Ry2 : S.Ry2,     me ? c.RAy : S.RAy,
                 me ? c.ratio : S.ratio, me ? c.invC : S.invC,   me ? c.invCc : S.invCc,
                 me ? c.dCx : S.dCx,     me ? c.dACx : S.dACx};
  }
  {
    const bool me = j == 4;
    const SegConst& c = I.iceseg;
    S = SegConst{me ? c.Tn : S.Tn,       me ? c.Ty2 : S.Ty2,     me ? c.TAy : S.TAy,
                 me ? c.Rn : S.Rn,       me ? c.Ry2 : S.Ry2,     me ? c.RAy : S.RAy,
                 me ? c.ratio : S.ratio, me ? c.invC : S.invC,   me ? c.invCc : S.invCc,
                 me ? c.dCx : S.dCx,     me ? c.dACx : S.dACx};
  }
  const bool air = j != 4;
  double v_unused;
  const Segment sg = segment_const(S, air ? M.A_air : M.A_ice, air ? A2 : A2i, sj, air, v_unused,
                                   tab);
#if AIRICE_RAY_STAMP
  ts[3] = __builtin_amdgcn_s_memtime() + (unsigned long long)(0.0 * (sg.thd + sg.t + sg.geo));
#endif
  // outputs that are functions of the chain's sines (every lane; lane 0 writes)
  const double inc = any ? k_asin(vinc) * M.r2d : 0.0;
  const double recv_ice = k_asin(sin_asin(I.iceseg.ratio * u_ice)) * M.r2d;
  double tS, tP;
  fresnel_from_sine(I.n_air_ice, I.n_ice0, I.n_ratio, vinc, tS, tP);
  double thd_air = 0.0, t_air = 0.0, geo_air = 0.0;
#pragma unroll
  for (int q = 0; q <= 3; ++q) {
    const double a = __shfl(sg.thd, q), b = __shfl(sg.t, q), c = __shfl(sg.geo, q);
    if (on[q]) {
      thd_air += a;
      t_air += b;
      geo_air += c;
    }
  }
  double thd_ice = 0.0, t_ice = 0.0, geo_ice = 0.0;
  {
    const double a = __shfl(sg.thd, 4), b = __shfl(sg.t, 4), c = __shfl(sg.geo, 4);
    if (on[4]) {
      thd_ice += a;
      t_ice += b;
      geo_ice += c;
    }
  }
#if AIRICE_RAY_STAMP
  ts[4] = __builtin_amdgcn_s_memtime() +
          (unsigned long long)(0.0 * (thd_air + thd_ice + t_air + t_ice + geo_air + geo_ice + tS +
                                      tP + inc + recv_ice));
#endif
  if (lane != 0) return;
  d[0] = 0;
  d[1] = H;
  d[2] = thd_air + thd_ice;
  d[3] = thd_air;
  d[4] = thd_ice;
  d[5] = (t_ice + t_air) * kSpeedC;
  d[6] = t_air * kSpeedC;
  d[7] = t_ice * kSpeedC;
  d[8] = (t_ice + t_air) * 1e9;
  d[9] = t_air * 1e9;
  d[10] = t_ice * 1e9;
  d[11] = theta;
  d[12] = inc;
  d[13] = in_ice ? recv_ice : 0.0;
  d[14] = tS;
  d[15] = tP;
  d[16] = geo_air;
  d[17] = geo_ice;
}

// One-ray launch (n = 1): one wave, ray_solution_wave, lane 0 writes dummy[0..17].
__global__ __launch_bounds__(64) void scalar_ray_kernel(DevMedium M, IceConsts I,
                                                        const double* __restrict__ launch,
                                                        const double* __restrict__ txh, int in_ice,
                                                        double* __restrict__ out, size_t ld,
                                                        Signal sig) {
  prefetch_kernargs<sizeof(DevMedium) + sizeof(IceConsts)>();
  unsigned long long ts[6] = {0, 0, 0, 0, 0, 0};
#if AIRICE_RAY_STAMP
  // debug: shader-clock stamps (entry, row constants, sine chain, segment, sums, stores) in
  // out[18..23], deltas from entry
  ts[0] = __builtin_amdgcn_s_memtime();
#endif
  const bool inl = sig.n_in >= 2;  // the inputs in the kernel arguments
  double d[18];
  ray_solution_wave(M, I, inl ? sig.in[0] : launch[0], inl ? sig.in[1] : txh[0], in_ice != 0, d,
                    &kLogTable[0][0], ts);
  if (threadIdx.x != 0) return;
#pragma unroll
  for (int c = 0; c < 18; ++c) out[c * ld] = d[c];
#if AIRICE_RAY_STAMP
  ts[5] = __builtin_amdgcn_s_memtime();
  for (int c = 1; c < 6; ++c) out[(17 + c) * ld] = (double)(ts[c] - ts[0]);
#endif
  signal_done(sig);
}

__global__ __launch_bounds__(kBlock) void rays_kernel(DevMedium M, IceConsts I,
                                                      const double* __restrict__ launch,
                                                      const double* __restrict__ txh, int in_ice,
                                                      long long n, double* __restrict__ out,
                                                      size_t ld, Signal sig) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  double d[18];
  const bool inl = sig.n_in >= 2;  // one-ray call: its inputs in the kernel arguments
  ray_solution(M, I, inl ? sig.in[0] : launch[k], inl ? sig.in[1] : txh[k], in_ice != 0, d);
#pragma unroll
  for (int c = 0; c < 18; ++c) out[c * ld + k] = d[c];
  if (k == 0) signal_done(sig);  // armed for one-ray calls only
}

// ---------------------------------------------------------------------------
// Minimizer: per-query air path (GetAirPropagationPar .cc:661-804 semantics: the first
// layer derives L, the lower layers reuse it, .cc:757-771).
// ---------------------------------------------------------------------------
struct AirPath {
  Endpoint tx;      // Tx height endpoint
  Endpoint iceair;  // air model at the (possibly depth-shifted) ice height
  Endpoint rtop;    // Rx endpoint of the top layer
  int top, bot;
};


__host__ __device__ __forceinline__ AirPath make_air_path(const DevMedium& M, double H, double ice) {
  AirPath P;
  P.top = top_layer(M, H);
  P.bot = bottom_layer(M, ice);
  P.tx = air_endpoint(M, H);
  P.iceair = air_endpoint(M, ice);
  P.rtop = pick(P.top == P.bot, P.iceair, stop_of(M, P.top));
  P.rtop = pick(P.rtop.x == P.tx.x, P.tx, P.rtop);  // zero-length top segment
  return P;
}

// sin of the receive angle of the first layer (GetLayerHitPointPar .cc:562-589).
__host__ __device__ __forceinline__ double first_layer_v2(const DevMedium& M, double n_tx, double n_rtop,
                                                 double theta) {
  const double v1 = sin_start((180 - theta) * M.d2r);
  return sin_asin((n_tx * sin_asin(v1)) / n_rtop);
}

// The four endpoint quantities fDnfR needs (prim_D): a bisection keeps only these in VGPRs.
struct Slim {
  double y2, Ay, Cx, invC;
};

__host__ __device__ __forceinline__ Slim slim(const Endpoint& p) { return Slim{p.y2, p.Ay, p.Cx, p.invC}; }

__host__ __device__ __forceinline__ Slim pick(bool c, const Slim& a, const Slim& b) {
  return Slim{c ? a.y2 : b.y2, c ? a.Ay : b.Ay, c ? a.Cx : b.Cx, c ? a.invC : b.invC};
}

// Slim air endpoint at x >= 0 (Tx heights and ice heights are non-negative; a negative x
// would need y(x) != n(|x|), handled by the full Endpoint path).
__host__ __device__ __forceinline__ Slim air_slim(const DevMedium& M, double x, double& n) {
  const double zabs = fabs(x);
  const int l = air_layer(M, zabs);
  const double B = sel5(M.B, l), C = sel5(M.negC, l);
  const double e_abs = exp(C * zabs);
  n = M.A_air + B * e_abs;
  const double y = (x >= 0.0) ? n : M.A_air + B * exp(C * x);
  return Slim{y * y, M.A_air * y, C * x, 1.0 / C};
}

__host__ __device__ __forceinline__ Slim stop_slim(const DevMedium& M, int l) {
  Slim r = slim(M.stop[0]);
  r = pick(l == 1, slim(M.stop[1]), r);
  r = pick(l == 2, slim(M.stop[2]), r);
  r = pick(l == 3, slim(M.stop[3]), r);
  return r;
}

// Start endpoint of air layer l (scalar reads when l is wave-uniform, as start_slim below).
__host__ __device__ __forceinline__ Endpoint start_endpoint(const DevMedium& M, int l) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int lu = __builtin_amdgcn_readfirstlane(l);
  if (__ballot(l != lu) == 0) return M.start[lu];
#endif
  Endpoint r = M.start[0];
  r = pick(l == 1, M.start[1], r);
  r = pick(l == 2, M.start[2], r);
  r = pick(l == 3, M.start[3], r);
  return r;
}

// Start end of air layer l: a scalar read when l is the same on every lane of the wave (a batch
// with one ice height), per-lane selects otherwise.
__host__ __device__ __forceinline__ Slim start_slim(const DevMedium& M, int l) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int lu = __builtin_amdgcn_readfirstlane(l);
  if (__ballot(l != lu) == 0) return slim(M.start[lu]);
#endif
  Slim r = slim(M.start[0]);
  r = pick(l == 1, slim(M.start[1]), r);
  r = pick(l == 2, slim(M.start[2]), r);
  r = pick(l == 3, slim(M.start[3]), r);
  return r;
}

__host__ __device__ __forceinline__ double stop_n(const DevMedium& M, int l) {
  double r = M.stop[0].n;
  r = (l == 1) ? M.stop[1].n : r;
  r = (l == 2) ? M.stop[2].n : r;
  r = (l == 3) ? M.stop[3].n : r;
  return r;
}


// fDnfR(R) - fDnfR(T) with one logarithm when both ends share C (identity (5)).
// tab: the log table (the roots kernel's LDS copy, else the global one).
__host__ __device__ __forceinline__ double delta_D(const Slim& T, const Slim& R, const RayL& RL,
                                          const double* tab = &kLogTable[0][0]) {
  const double syR = fast_sqrt(R.y2 - RL.LL), syT = fast_sqrt(T.y2 - RL.LL);
  const double d1 = log_ratio(R.Ay - RL.LL + RL.sAL * syR, T.Ay - RL.LL + RL.sAL * syT, tab);
  return (RL.L * R.invC) * RL.rsAL * ((R.Cx - T.Cx) - d1);
}

// Per-query state of the root finder (MinforLAng_params + the air path's endpoints).
struct Query {
  Slim tx, rtop, iceair, rx;
  double n_tx, n_rtop;
  double ratio;  // n_tx / n_rtop: the first layer's Snell step (as the table's SegConst::ratio)
  int top, bot;
  double dist;
  double depth_pos;  // MinforLAng_params.antennadepth (> 0 in ice, 0 in air)
};

// Sum of per-layer horizontal distances in air for launch angle theta (THD only: the time
// and geometric-path terms do not enter f).  Returns L0 through the reference.
__host__ __device__ __forceinline__ double air_thd(const DevMedium& M, const Query& q, double theta,
                                          double& L0, const double* tab) {
  if (q.top < q.bot) {  // no layer: the reference reads unset output slots (UB)
    L0 = __builtin_nan("");
    return 0.0;
  }
  // first_layer_v2 with the per-query ratio and the start-angle polynomial (theta in [90, 180]
  // here; other angles go through ocml's sin inside sin_start)
  const double v1 = sin_start((180 - theta) * M.d2r);
  const double L = q.n_rtop * sin_asin(q.ratio * sin_asin(v1));
  L0 = L;
  const RayL RL = ray_L(M.A_air * M.A_air, L);
  // The reference's layer loop (top -> bot) in three parts with the same summation order: the
  // Tx layer (both ends per query), the layers strictly between (both ends layer bounds: uniform
  // across the wave, read as scalars, no per-lane selects; at most layers 2 and 1), the ice layer
  // (start bound of the lowest layer -> the query's ice endpoint).
  double thd = 0.0;
  {
    double x1 = delta_D(q.tx, q.rtop, RL, tab);
    x1 *= -1;
    thd += x1;
  }
#pragma unroll
  for (int il = kMaxLayers - 2; il >= 1; --il) {
    if (il < q.top && il > q.bot) {
      double x1 = delta_D(slim(M.start[il]), slim(M.stop[il]), RL, tab);
      x1 *= -1;
      thd += x1;
    }
  }
  if (q.top > q.bot) {
    double x1 = delta_D(start_slim(M, q.bot), q.iceair, RL, tab);
    x1 *= -1;
    thd += x1;
  }
  return thd;
}

// delta_D at two ray parameters (two launch angles) on the same segment: the two chains in one
// straight-line block, so each hides the other's latency; every value as delta_D forms it.
__host__ __device__ __forceinline__ void delta_D2(const Slim& T, const Slim& R, const RayL& Ra,
                                         const RayL& Rb, const double* tab, double& xa,
                                         double& xb) {
  const double syRa = fast_sqrt(R.y2 - Ra.LL), syTa = fast_sqrt(T.y2 - Ra.LL);
  const double syRb = fast_sqrt(R.y2 - Rb.LL), syTb = fast_sqrt(T.y2 - Rb.LL);
  double da, db;
  log_ratio2(R.Ay - Ra.LL + Ra.sAL * syRa, T.Ay - Ra.LL + Ra.sAL * syTa,
             R.Ay - Rb.LL + Rb.sAL * syRb, T.Ay - Rb.LL + Rb.sAL * syTb, tab, da, db);
  xa = (Ra.L * R.invC) * Ra.rsAL * ((R.Cx - T.Cx) - da);
  xb = (Rb.L * R.invC) * Rb.rsAL * ((R.Cx - T.Cx) - db);
}

// MinimizeforLaunchAngle's THD in air and in the ice at two angles (the root finder's bracket
// ends f(lo), f(hi)), as air_thd + the ice term of solve_root's evaluation site computes each:
// the same operations in the same order per angle, the two angles' chains interleaved.
__host__ __device__ __forceinline__ void eval_thd2(const DevMedium& M, const IceConsts& I, const Query& q,
                                          double ta, double tb, const double* tab,
                                          double& air_a, double& ice_a, double& air_b,
                                          double& ice_b) {
  double La = __builtin_nan(""), Lb = __builtin_nan("");
  air_a = 0.0;
  air_b = 0.0;
  if (q.top >= q.bot) {
    const double v1a = sin_start((180 - ta) * M.d2r);
    const double v1b = sin_start((180 - tb) * M.d2r);
    La = q.n_rtop * sin_asin(q.ratio * sin_asin(v1a));
    Lb = q.n_rtop * sin_asin(q.ratio * sin_asin(v1b));
    const RayL Ra = ray_L(M.A_air * M.A_air, La), Rb = ray_L(M.A_air * M.A_air, Lb);
    double xa, xb;
    delta_D2(q.tx, q.rtop, Ra, Rb, tab, xa, xb);
    xa *= -1;
    xb *= -1;
    air_a += xa;
    air_b += xb;
#pragma unroll
    for (int il = kMaxLayers - 2; il >= 1; --il) {
      if (il < q.top && il > q.bot) {
        delta_D2(slim(M.start[il]), slim(M.stop[il]), Ra, Rb, tab, xa, xb);
        xa *= -1;
        xb *= -1;
        air_a += xa;
        air_b += xb;
      }
    }
    if (q.top > q.bot) {
      delta_D2(start_slim(M, q.bot), q.iceair, Ra, Rb, tab, xa, xb);
      xa *= -1;
      xb *= -1;
      air_a += xa;
      air_b += xb;
    }
  }
  ice_a = 0;
  ice_b = 0;
  if (q.depth_pos != 0) {
    const RayL Ra = ray_L(M.A_ice * M.A_ice, La), Rb = ray_L(M.A_ice * M.A_ice, Lb);
    double xa, xb;
    delta_D2(slim(I.ice0), q.rx, Ra, Rb, tab, xa, xb);
    ice_a += xa;
    ice_b += xb;
  }
}

// Two evaluations of f spread over a wave, for one-query calls (scalar_solve_kernel): lanes 0-4
// take the Tx layer, layers 2 and 1 (when strictly between), the ice layer and the segment in the
// ice at theta_a, lanes 32-36 the same at theta_b, each with the same delta_D as air_thd, and the
// sums are formed in air_thd's order from the lanes' values -- the same bits as the one-lane
// evaluation, with ~1/4 of its dependent chain.  Every lane holds the same query, so everything
// else stays wave-uniform.
__device__ __forceinline__ void eval_thd_wave(const DevMedium& M, const IceConsts& I,
                                              const Query& q, double theta_a, double theta_b,
                                              const double* tab, double& thd_air_a,
                                              double& thd_ice_a, double& thd_air_b,
                                              double& thd_ice_b) {
  const int lane = (int)(threadIdx.x & 31);
  const double theta = (threadIdx.x & 32) ? theta_b : theta_a;
  const bool air = q.top >= q.bot;
  double L = __builtin_nan("");
  if (air) {
    const double v1 = sin_start((180 - theta) * M.d2r);
    L = q.n_rtop * sin_asin(q.ratio * sin_asin(v1));
  }
  const bool ice = lane == 4;
  const RayL RL = ray_L(ice ? M.A_ice * M.A_ice : M.A_air * M.A_air, L);
  Slim T = q.tx, R = q.rtop;  // lane 0 (and the lanes past 4, whose value is unused)
  T = pick(lane == 1, slim(M.start[2]), T);
  R = pick(lane == 1, slim(M.stop[2]), R);
  T = pick(lane == 2, slim(M.start[1]), T);
  R = pick(lane == 2, slim(M.stop[1]), R);
  T = pick(lane == 3, slim(M.start[0]), T);
  T = pick(lane == 3 && q.bot >= 1, slim(M.start[1]), T);
  T = pick(lane == 3 && q.bot >= 2, slim(M.start[2]), T);
  T = pick(lane == 3 && q.bot >= 3, slim(M.start[3]), T);
  R = pick(lane == 3, q.iceair, R);
  T = pick(ice, slim(I.ice0), T);
  R = pick(ice, q.rx, R);
  const double x = delta_D(T, R, RL, tab);
  auto sums = [&](int l0, double& thd_air, double& thd_ice) {
    const double d0 = __shfl(x, l0), d1 = __shfl(x, l0 + 1), d2 = __shfl(x, l0 + 2),
                 d3 = __shfl(x, l0 + 3), d4 = __shfl(x, l0 + 4);
    thd_air = 0.0;
    if (air) {
      thd_air += -d0;
      if (2 < q.top && 2 > q.bot) thd_air += -d1;
      if (1 < q.top && 1 > q.bot) thd_air += -d2;
      if (q.top > q.bot) thd_air += -d3;
    }
    thd_ice = 0;
    if (q.depth_pos != 0) thd_ice += d4;
  };
  sums(0, thd_air_a, thd_ice_a);
  sums(32, thd_air_b, thd_ice_b);
}

// ---------------------------------------------------------------------------
// Air2IceRayTracing (.cc:1464-1616) in two launches: stage 1 finds the launch angle
// (bracket, probe, bisection) keeping only the slim per-query state live; stage 2 rebuilds
// the full endpoints and evaluates every output at the root.  Splitting keeps the
// register-hungry full evaluation out of the bisection kernel's allocation.  Stage 1 parks
// the root and status in output slots that stage 2 overwrites.
// ---------------------------------------------------------------------------
struct Geometry {
  double H, D, ice, depth;  // after the Rx-in-air shift (.cc:1472-1479)
  double depth_pos;         // MinforLAng_params.antennadepth
};

__host__ __device__ __forceinline__ Geometry shift(double H, double D, double ice, double depth) {
  Geometry g;
  g.H = H;
  g.D = D;
  if (depth >= 0) {
    g.ice = depth + ice;
    g.depth = 0;
    g.depth_pos = 0;
  } else {
    g.ice = ice;
    g.depth = depth;
    g.depth_pos = -depth;
  }
  return g;
}

// What the root finder returns for one query.
struct SolveResult {
  double root;
  int status;
  int n_eval, n_est, n_inside;  // evaluations: all, secant search, bisection midpoints (stats)
#if AIRICE_SCALAR_STAMP
  int t_setup = 0, t_lean = 0;  // debug: shader clocks of the set-up and of the lean bisection runs
  int t_pre = 0, t_post = 0;    //        loop top -> evaluation, evaluation -> loop top
#endif
#if AIRICE_ROOTS_STAMP == 3
  int tb[6] = {0, 0, 0, 0, 0, 0};
#endif
#if AIRICE_ROOTS_STAMP == 2
  int t_next = 0, t_eval = 0;  // debug: shader clocks in next_point and in the evaluations
  int t_upd = 0, t_pre = 0;    //        in update, and before the loop (set-up, paired ends)
  int t_begin = 0;             //        in the set-up (begin)
#endif
};

enum { PH_PROBE = 0, PH_FLO = 1, PH_FHI = 2, PH_EST = 3, PH_G1 = 4, PH_G2 = 5, PH_BISECT = 6,
       PH_DONE = 7 };

#if AIRICE_SORTED_STATS
// debug build: wave-level executions of the root finder's blocks (tools/solve_blocks.py): the
// first active lane of each execution counts it, so a block that several lanes of a wave run
// together counts once -- the count of the wave's instruction streams through it (device code
// only: the host form of the root finder counts nothing)
__device__ unsigned long long g_dbg_exec[16];
#endif
#if AIRICE_SORTED_STATS && defined(__HIP_DEVICE_COMPILE__)
#define DBG_EXEC(i)                                                                 \
  do {                                                                              \
    if ((int)(threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) atomicAdd(&g_dbg_exec[i], 1ull); \
  } while (0)
#else
#define DBG_EXEC(i) \
  do {              \
  } while (0)
#endif

// Shader clock for the debug stamp builds (0 on the host pass of the shared code).
__host__ __device__ __forceinline__ unsigned long long dbg_clock() {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_s_memtime();
#else
  return 0;
#endif
}

// Quotients and the first guess's tangent that only steer the search (the root comes from GSL's
// bisection replay): v_rcp_f64 (~2^-24 relative) and the fast single-precision tangent on the
// device, the plain forms on the host.
__host__ __device__ __forceinline__ double rcp_steer(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcp(x);
#else
  return 1.0 / x;
#endif
}
// isfinite / isnan as each pass has them (ocml's on the device: the kernels' code is unchanged)
__host__ __device__ __forceinline__ bool k_isfinite(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return isfinite(x);
#else
  return std::isfinite(x);
#endif
}
__host__ __device__ __forceinline__ bool k_isnan(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return isnan(x);
#else
  return std::isnan(x);
#endif
}
__host__ __device__ __forceinline__ float tanf_steer(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __tanf(x);
#else
  return std::tan(x);
#endif
}

// The air model at the ice height of a batch whose queries share it (the ice end of every air
// path), formed once per block by the kernel: x the ice height it is for, bot its layer.
struct IceAirPre {
  Slim s;
  double n, x;
  int bot;
};

// The root finder of one query as a state machine with a single evaluation site (RootSearch):
// begin() sets up the bracket and the probe, next_point() runs the evaluation-free bisection
// steps and returns the point to evaluate next, update() takes f there.  solve_root() below drives
// one query to its root.
struct RootSearch {
  Query q;
  double lo, hi;
  double f_lower, f_upper;
  double tau;
  // Sign guards.  f(theta) = D - THD(theta) is monotone in theta wherever it is finite, so
  // between two exactly evaluated points with the same sign and |f| >= tau (far above the
  // evaluation's rounding noise) every point has that sign.  gL / gR: the innermost evaluated
  // points with the sign of f(lo) / f(hi); okL / okR: |f(lo)| / |f(hi)| >= tau, so the guard
  // regions [lo, gL] / [gR, hi] are safe.  A secant search finds the root, two guards straddle
  // it, and the bisection then evaluates f only at midpoints between the guards: the same
  // midpoints, signs and root as evaluating every one (tests/test_gpu_bisect_replay.py checks
  // this bit for bit against AIRICE_BISECT_EXACT=1).
  double gL, fL, gR, fR;  // fL holds f(lo) between PH_FLO and PH_FHI
  // secant search for the root: the first step in u = tan(180 - theta), where THD is close to
  // linear (a straight ray's is exactly H u; single precision is plenty for a first guess), then
  // steps on the last points (x1, f1), (x2, f2) and, from the second search point on, inverse
  // quadratic interpolation through (x0, f0) as well (the secant step plus a curvature term).
  // PH_G1/G2: guards at x2 -/+ dlt, where x2 is the search's last point (it stays put after the
  // search) and dlt lives in x1 (dead once the search ends).
  double x0, f0, x1, f1, x2, f2;
  int phase, status, iter, est, n_eval, n_inside;
  bool root_zero;  // the failed probe reports root 0 (.cc:1500-1509)
  bool okL, okR, exact;
#if AIRICE_SCALAR_STAMP
  int t_lean;
#endif
#if AIRICE_ROOTS_STAMP == 3
  int tb[6];  // debug: set-up stamps (tx endpoint, ice endpoint + rtop, ratio, rx, probe, total)
#endif

  __host__ __device__ __forceinline__ double& dlt() { return x1; }

  // Air2IceRayTracing's set-up (.cc:1487-1509): the query's endpoints, the bracket [thR - 16, thR]
  // and the 0.05-degree probe.  An uninitialised solver state (non-finite bracket end) is modelled
  // as zeros.
  __host__ __device__ __forceinline__ void begin(const DevMedium& M, const IceConsts& I, const Geometry& g,
                                        double thR, bool exact_,
                                        const IceAirPre* pre = nullptr) {
#if AIRICE_ROOTS_STAMP == 3
    const unsigned long long tb0 = dbg_clock();
#endif
    status = 0;
    exact = exact_;
#if AIRICE_SCALAR_STAMP
    t_lean = 0;
#endif
    q.depth_pos = g.depth_pos;
    q.dist = g.D;
    q.top = top_layer(M, g.H);
    // the ice end: the block's copy when every lane of the wave has the batch's ice height
    bool have_pre = false;
    if (pre != nullptr) {
#if defined(__HIP_DEVICE_COMPILE__)
      have_pre = __ballot(g.ice != pre->x) == 0;
#else
      have_pre = g.ice == pre->x;
#endif
    }
    double n_ice;
    if (have_pre) {
      q.bot = pre->bot;
      q.iceair = pre->s;
      n_ice = pre->n;
    } else {
      q.bot = bottom_layer(M, g.ice);
      q.iceair = air_slim(M, g.ice, n_ice);
    }
    q.tx = air_slim(M, g.H, q.n_tx);
#if AIRICE_ROOTS_STAMP == 3
    tb[0] = (int)(dbg_clock() + (unsigned long long)(0.0 * (q.tx.y2 + q.n_tx)) - tb0);
#endif
    // Rx end of the top layer: the ice, or the layer's lower boundary (stop endpoint)
    const bool to_ice = q.top == q.bot;
    q.rtop = pick(to_ice, q.iceair, stop_slim(M, q.top));
    q.n_rtop = to_ice ? n_ice : stop_n(M, q.top);
    const double x_rtop = to_ice ? g.ice : sel5(M.atm, q.top);
    if (x_rtop == g.H) {  // zero-length top segment (see segment())
      q.rtop = q.tx;
      q.n_rtop = q.n_tx;
    }
#if AIRICE_ROOTS_STAMP == 3
    tb[1] = (int)(dbg_clock() + (unsigned long long)(0.0 * (q.rtop.y2 + q.n_rtop)) - tb0);
#endif
    q.ratio = q.n_tx / q.n_rtop;
#if AIRICE_ROOTS_STAMP == 3
    tb[2] = (int)(dbg_clock() + (unsigned long long)(0.0 * q.ratio) - tb0);
#endif
    {
      const double e = exp(M.negC_ice * g.depth_pos);
      const double y = M.A_ice + M.B_ice * e;
      // 1/C of the ice from the host-folded surface endpoint (the same IEEE quotient): a kernel
      // argument, so it occupies no VGPRs across the loop
      q.rx = Slim{y * y, M.A_ice * y, M.negC_ice * g.depth_pos, I.ice0.invC};
    }
#if AIRICE_ROOTS_STAMP == 3
    tb[3] = (int)(dbg_clock() + (unsigned long long)(0.0 * q.rx.y2) - tb0);
#endif
    lo = thR - 16;
    hi = thR;
    phase = PH_FLO;
    bool probe_bad = false;  // the probe ended with lo > hi: the reference then reports root 0
    if (M.const_air) lo = 90;  // pythonwrapper constant air index: [90, thR], no probe (.cc:978-980)
    if (!M.const_air && lo < 90.001) {
      lo = 90.001;
      phase = PH_PROBE;
      // While n(Tx) sin(180-lo) exceeds 1 by a margin (1e-6) the ray parameter L > A_air = 1,
      // so sqrt(A^2-L^2) and THD are NaN whatever the rounding: those probe steps need no
      // evaluation (.cc:1496-1509 would reject each of them).
      if (q.top >= q.bot) {
        const double thr = 180 - asin((1 + 1e-6) / q.n_tx) * M.r2d;  // NaN if n(Tx) < 1+1e-6
        // while (lo < thr && !(lo > hi - 0.1)) lo = lo + 0.05, in closed form (airice_lean.hpp)
        bool stepped;
        lo = probe_steps(lo, 0.05, hi - 0.1, thr, true, stepped);
        if (stepped) status |= AIRICE_SOLVE_PROBED;
      } else {
        // no air layer (Tx above the atmosphere, e.g. the table lookup's x100 fallback): THD in
        // air is 0 at every angle, so the probe only stops at lo > hi - 0.1 -- up to ~900 steps
        // whose outcome needs no evaluation, taken in closed form (airice_lean.hpp)
        bool stepped;
        lo = probe_steps(lo, 0.05, hi - 0.1, 0.0, false, stepped);
        if (stepped) status |= AIRICE_SOLVE_PROBED;
        if (hi < 90.001 && hi > 90.00) hi = 90.05;
        phase = PH_FLO;
        if (lo > hi) {
          status |= AIRICE_SOLVE_BAD_BRACKET;
          probe_bad = true;
          phase = PH_DONE;
        }
      }
    } else {
      if (hi < 90.001 && hi > 90.00) hi = 90.05;
      if (lo > hi) {  // gsl_root_fsolver_set: EINVAL, nothing initialised
        status |= AIRICE_SOLVE_BAD_BRACKET;
        phase = PH_DONE;
      }
    }
    // GSL's reported root is 0.5 (lo + hi) of the final bracket on every path (each iterate sets
    // it so, and the exact-zero exits make lo == hi), except the failed probe, which reports 0:
    // the root is formed once at the end instead of being carried through the loop
#if AIRICE_ROOTS_STAMP == 3
    tb[4] = (int)(dbg_clock() + (unsigned long long)(0.0 * (lo + hi)) - tb0);
    tb[5] = phase == PH_PROBE || (status & AIRICE_SOLVE_PROBED) ? 1 : 0;
#endif
    root_zero = probe_bad;
    f_lower = 0.0;
    f_upper = 0.0;
    iter = 0;
    tau = 1e-6 + 1e-10 * fabs(g.D);
    okL = false;
    okR = false;
    gL = fL = gR = fR = 0.0;
    x0 = f0 = x1 = f1 = x2 = f2 = 0.0;
    est = 0;
    n_eval = 0;
    n_inside = 0;
  }

  __host__ __device__ __forceinline__ void guard(double x, double f) {
    if (!(fabs(f) >= tau) || !(x > gL && x < gR)) return;
    if ((f < 0.0) == (fL < 0.0)) {
      gL = x;
      fL = f;
    } else {
      gR = x;
      fR = f;
    }
  }

  // gsl_root_test_interval(lo, hi, 0, 1e-9) and the driver's max_iter (.cc:355-371)
  __host__ __device__ __forceinline__ void finish(bool frozen) {
    const double tol = 0.000000001;
    bool cont;
    if (lo > hi) {
      cont = false;
    } else {
      const double min_abs = ((lo > 0.0 && hi > 0.0) || (lo < 0.0 && hi < 0.0))
                                 ? (fabs(lo) < fabs(hi) ? fabs(lo) : fabs(hi))
                                 : 0.0;
      const double tolerance = 0 + tol * min_abs;
      cont = !(fabs(hi - lo) < tolerance);
    }
    if (cont && iter == 40) status |= AIRICE_SOLVE_MAXITER;
    if (frozen || !cont || iter == 40) phase = PH_DONE;
  }

  // gsl_root_fsolver_set's second end, f(hi) (fL holds f(lo)): the bracket state, the guards and
  // the secant search's first guess
  __host__ __device__ __forceinline__ void on_fhi(const DevMedium& M, double f) {
    phase = PH_BISECT;
    if (!k_isfinite(f)) {
      status |= AIRICE_SOLVE_NONFINITE_END;
    } else {
      f_lower = fL;
      f_upper = f;
      if (!exact) {
        gL = lo;
        gR = hi;
        fR = f;
        okL = fabs(fL) >= tau;
        okR = fabs(fR) >= tau;
        if (okL && okR) {
          if ((fL < 0.0) == (fR < 0.0)) {
            gL = hi;  // no sign change: every midpoint has the ends' sign
          } else {
            const float ul = tanf_steer((float)((180 - lo) * M.d2r));
            const float uh = tanf_steer((float)((180 - hi) * M.d2r));
            const float un = uh - (float)fR * ((uh - ul) / (float)(fR - fL));
            x1 = hi;
            f1 = fR;
            x0 = lo;
            f0 = fL;
            x2 = 180 - (double)atanf(un) * M.r2d;  // first guess, evaluated first
            phase = PH_EST;
          }
        }
      }
    }
  }

  // f(lo) and f(hi) in one pass (eval_thd2: two independent chains per lane, ~1.3x the time of one
  // evaluation instead of 2x); a lane that is probing reaches PH_FLO in the loop and evaluates the
  // ends there
  __host__ __device__ __forceinline__ void ends_paired(const DevMedium& M, const IceConsts& I,
                                              const double* tab) {
    if (phase != PH_FLO) return;
    double air_a, ice_a, air_b, ice_b;
    eval_thd2(M, I, q, lo, hi, tab, air_a, ice_a, air_b, ice_b);
    const double fa = (q.dist - (ice_a + air_a));
    ++n_eval;
    if (!k_isfinite(fa)) {
      status |= AIRICE_SOLVE_NONFINITE_END;
      phase = PH_BISECT;
    } else {
      fL = fa;
      ++n_eval;
      on_fhi(M, q.dist - (ice_b + air_b));
    }
  }

  // The evaluation-free bisection steps and the next point to evaluate.  False: the query is done
  // (phase PH_DONE) without another evaluation.
  __host__ __device__ __forceinline__ bool next_point(const DevMedium& M, double& x) {
    const double tol = 0.000000001;
    if (phase == PH_BISECT) {
      DBG_EXEC(1);
      // steps that need no evaluation: an exact zero at a bracket end (GSL returns that end),
      // or a midpoint inside a guard region, whose sign is the region's: lo (left) or hi
      // (right) moves to it, as gsl_root_fsolver_iterate would
      if (f_lower == 0.0 || f_upper == 0.0) {
        ++iter;
        const double r0 = (f_lower == 0.0) ? lo : hi;
        lo = r0;
        hi = r0;
        finish(false);
        phase = PH_DONE;  // lo == hi: gsl_root_test_interval converges
        return false;
      }
      if ((okL || okR) && lo > 0.0) {
#if AIRICE_SCALAR_STAMP
        const unsigned long long tl0 = dbg_clock();
#endif
        // lean run (0 < lo < hi here): the root GSL reports after a step is 0.5 (lo + hi) of the
        // new bracket either way; the interval test reduces to hi - lo < tol lo
        const double gl = okL ? gL : -1.0, gr = okR ? gR : __builtin_inf();
        const double lo0 = lo, hi0 = hi;
        bool done = false;
        DBG_EXEC(2);
        // the whole run in closed form when its midpoints are exact (airice_lean.hpp: every
        // bracket the probe did not move), the same lo, hi, steps and exit as the steps below
        LeanRun lr;
        if (lean_closed(lo, hi, iter, gL, gR, okL, okR, tol, lr)) {
          DBG_EXEC(13);
          lo = lr.lo;
          hi = lr.hi;
          iter += lr.steps;
          status = lr.maxiter ? (status | AIRICE_SOLVE_MAXITER) : status;
          done = lr.done;
        } else {
          // the steps as selects, four per trip, so that the chain is midpoint -> compare ->
          // select without a divergent exit per step
          bool stop = false;
          while (!stop) {
            DBG_EXEC(3);
#pragma unroll
            for (int u = 0; u < kLeanUnroll; ++u) {
              const double xm = (lo + hi) / 2.0;
              const bool inL = xm <= gl, inR = !inL && xm >= gr;
              const bool mv = !stop && (inL || inR);  // otherwise: evaluate this midpoint
              lo = (mv && inL) ? xm : lo;
              hi = (mv && inR) ? xm : hi;
              iter += mv ? 1 : 0;
              const bool cont = !(fabs(hi - lo) < 0 + tol * lo);
              const bool fin = mv && (!cont || iter == 40);
              status = (fin && cont) ? (status | AIRICE_SOLVE_MAXITER) : status;
              done = done || fin;
              stop = stop || !mv || fin;
            }
          }
        }
        if (lo != lo0) f_lower = fL;
        if (hi != hi0) f_upper = fR;
#if AIRICE_SCALAR_STAMP
        t_lean += (int)(dbg_clock() - tl0) + (int)(0.0 * (lo + hi));
#endif
        if (done) {
          phase = PH_DONE;
          return false;
        }
      }
    }
    if (phase == PH_FHI) {
      x = hi;
    } else if (phase == PH_BISECT) {
      x = (lo + hi) / 2.0;
    } else if (phase == PH_EST) {
      DBG_EXEC(11);
      // the secant point only steers the search (the root comes from GSL's bisection replay), so
      // its quotient takes v_rcp_f64 (~2^-24 relative) instead of the IEEE division
      x = (est == 0) ? x2 : x2 - f2 * ((x2 - x1) * rcp_steer(f2 - f1));
      // theta(f) through (x0, f0), (x1, f1), (x2, f2) in Newton form, at f = 0: the secant step
      // minus f1 f2 times the second divided difference (the search only steers; a point outside
      // the guards falls back to their midpoint below)
      if (est >= 1) {
        const double d1 = (x2 - x1) * rcp_steer(f2 - f1);
        const double d0 = (x1 - x0) * rcp_steer(f1 - f0);
        x += f1 * f2 * ((d1 - d0) * rcp_steer(f2 - f0));
      }
      if (!(x > gL && x < gR)) x = 0.5 * (gL + gR);  // safeguard: the guards' midpoint
    } else if (phase == PH_G1) {
      x = x2 - dlt();
    } else if (phase == PH_G2) {
      x = x2 + dlt();
    } else {
      x = lo;
    }
    return true;
  }

  // f = D - THD at x, the point next_point() returned.  REUSE_PROBE: a probing lane's last probe
  // evaluation (at x = lo, the point gsl_root_fsolver_set evaluates next) is taken as f(lo).
  template <bool REUSE_PROBE>
  __host__ __device__ __forceinline__ void update(const DevMedium& M, double x, double thd_air,
                                         double thd_ice) {
    ++n_eval;
    n_inside += (phase == PH_BISECT);
    const double f = (q.dist - (thd_ice + thd_air));
    if (phase == PH_PROBE) {
      DBG_EXEC(5);
      if ((!k_isnan(thd_air) && thd_air > 0) || lo > hi - 0.1) {
        if (hi < 90.001 && hi > 90.00) hi = 90.05;
        phase = PH_FLO;
        if (lo > hi) {
          status |= AIRICE_SOLVE_BAD_BRACKET;
          root_zero = true;
          phase = PH_DONE;
        } else if (REUSE_PROBE) {
          // this trip evaluated f at x = lo, the point gsl_root_fsolver_set evaluates next
          // (f(lo)): the same point and arithmetic, so its value is PH_FLO's result and the lane
          // goes on to f(hi) one trip earlier
          if (!k_isfinite(f)) {
            status |= AIRICE_SOLVE_NONFINITE_END;
            phase = PH_BISECT;
          } else {
            fL = f;
            phase = PH_FHI;
          }
        }
      } else {
        lo = lo + 0.05;
        status |= AIRICE_SOLVE_PROBED;
      }
    } else if (phase == PH_FLO) {
      DBG_EXEC(6);
      if (!k_isfinite(f)) {
        status |= AIRICE_SOLVE_NONFINITE_END;
        phase = PH_BISECT;
      } else {
        fL = f;
        phase = PH_FHI;
      }
    } else if (phase == PH_FHI) {
      DBG_EXEC(7);
      on_fhi(M, f);
    } else if (phase == PH_EST) {
      DBG_EXEC(8);
      if (est > 0) {
        x0 = x1;
        f0 = f1;
        x1 = x2;
        f1 = f2;
      }
      x2 = x;
      f2 = f;
      ++est;
      if (!k_isfinite(f)) {
        phase = PH_BISECT;
      } else if (fabs(f) < tau) {
        // at the root: guards a few tau either side, scaled by the local secant slope
        const double sl = (x2 - x1) * rcp_steer(f2 - f1);  // dtheta / df
        const double a = (x2 - x1) * (f1 - f0), b = (x1 - x0) * (f2 - f1);  // (before dlt takes x1)
        dlt() = 4.0 * tau * fabs(sl);
        const bool room = dlt() > 0.0 && dlt() < (gR - gL);
        // x1 is a search point near the root (est >= 2), so the secant slope through it is the
        // local one, and f at x2 -+ dlt is f2 -+ 4 tau sign(sl) to first order: |.| >= 3 tau with
        // the root between.  The guards then take those signs without evaluating f there -- when
        // the slope is consistent: the previous secant slope (x0, x1) has the same sign and is
        // within 2x of it (sl (f2 - f1) = x2 - x1 and its twin, compared as products: no
        // quotient, and any NaN fails), so f's curvature cannot have moved the root out of
        // [x2 - dlt, x2 + dlt].  Otherwise, and for the first search point (x1 is the bracket
        // end), both guards are evaluated (a side whose guard already lies at the root needs none).
        const bool consistent = a * b > 0.0 && fabs(a) <= 2.0 * fabs(b) && fabs(b) <= 2.0 * fabs(a);
        if (room && est >= 2 && (AIRICE_NO_CHECK || consistent)) {
          const double fm = sl > 0.0 ? -tau : tau;  // f(x2 - dlt)
          guard(x2 - dlt(), fm);
          guard(x2 + dlt(), -fm);
          phase = PH_BISECT;
        } else {
          const bool needL = !(x2 - gL <= 0.0), needR = !(gR - x2 <= 0.0);
          phase = room ? (needL ? PH_G1 : (needR ? PH_G2 : PH_BISECT)) : PH_BISECT;
        }
      } else {
        guard(x, f);
        if (est >= 12) phase = PH_BISECT;
      }
    } else if (phase == PH_G1 || phase == PH_G2) {
      DBG_EXEC(9);
      if (k_isfinite(f)) guard(x, f);
      phase = phase == PH_G1 ? PH_G2 : PH_BISECT;
    } else {  // PH_BISECT: gsl_root_fsolver_iterate at a midpoint between the guards
      DBG_EXEC(10);
      if (!exact && k_isfinite(f)) guard(x, f);
      ++iter;
      bool frozen = false;
      if (!k_isfinite(f)) {
        // EBADFUNC leaves the state unchanged: every later iterate repeats this one, so the
        // driver ends at max_iter with the same root.
        status |= AIRICE_SOLVE_STALE_MID | AIRICE_SOLVE_MAXITER;
        frozen = true;
      } else if (f == 0.0) {
        lo = x;
        hi = x;
      } else if ((f_lower > 0.0 && f < 0.0) || (f_lower < 0.0 && f > 0.0)) {
        hi = x;
        f_upper = f;
      } else {
        lo = x;
        f_lower = f;
      }
      finish(frozen);
    }
  }

  __host__ __device__ __forceinline__ double root() const { return root_zero ? 0.0 : 0.5 * (lo + hi); }
};

// MinimizeforLaunchAngle's f terms at theta (.cc:873-917): THD in air and in the ice.
__host__ __device__ __forceinline__ void eval_thd(const DevMedium& M, const IceConsts& I, const Query& q,
                                         double theta, const double* tab, double& thd_air,
                                         double& thd_ice) {
  double L;
  thd_air = air_thd(M, q, theta, L, tab);
  thd_ice = 0;
  if (q.depth_pos != 0) {
    const RayL RL = ray_L(M.A_ice * M.A_ice, L);
    thd_ice += delta_D(slim(I.ice0), q.rx, RL, tab);
  }
}

// Root finding of Air2IceRayTracing (.cc:1487-1521): the probe loop, gsl_root_fsolver_set and the
// FindFunctionRoot driver (.cc:340-374) with gsl_root_fsolver_bisection +
// gsl_root_test_interval(lo, hi, 0, 1e-9) semantics, as one per-lane state machine with a single
// evaluation site: lanes that are probing, setting up the bracket or bisecting share each
// evaluation instead of waiting for each other (the probe runs in ~7% of queries).
// WAVE: one query per wave (scalar_solve_kernel), each evaluation spread over the lanes.
template <bool WAVE = false>
__host__ __device__ __forceinline__ SolveResult solve_root(const DevMedium& M, const IceConsts& I,
                                                  const Geometry& g, double thR, bool exact,
                                                  const double* tab,
                                                  const IceAirPre* pre = nullptr) {
#if AIRICE_SCALAR_STAMP
  const unsigned long long ts0 = dbg_clock();
#endif
#if AIRICE_ROOTS_STAMP == 2
  const unsigned long long ts_entry = dbg_clock();
#endif
  RootSearch s;
  s.begin(M, I, g, thR, exact, pre);
#if AIRICE_ROOTS_STAMP == 2
  const unsigned long long ts_begun = dbg_clock() + (unsigned long long)(0.0 * (s.lo + s.hi + s.q.ratio));
#endif
  if constexpr (!WAVE) s.ends_paired(M, I, tab);
#if AIRICE_SCALAR_STAMP
  const int t_setup = (int)(dbg_clock() - ts0) + (int)(0.0 * (s.lo + s.hi));
  int t_pre = 0, t_post = 0;
  unsigned long long tq = dbg_clock();
#endif
  // WAVE: f(lo) and f(hi), and the two guards, are independent pairs of points; the wave evaluates
  // each pair at once and keeps the second value for the next trip (the same points, the same
  // bits, two sequential evaluations fewer)
  bool have_next = false;
  double next_air = 0.0, next_ice = 0.0;
#if AIRICE_ROOTS_STAMP == 2
  int rs_next = 0, rs_eval = 0, rs_upd = 0;
  const unsigned long long rs_l0 = dbg_clock() + (unsigned long long)(0.0 * (s.lo + s.hi));
#endif
  while (s.phase != PH_DONE) {
    DBG_EXEC(0);
    if constexpr (WAVE) {
      // one query per wave: the phase and the counters are the same on every lane; scalar copies
      // let the phase dispatch branch on SCC instead of exec masks
      s.phase = __builtin_amdgcn_readfirstlane(s.phase);
      s.est = __builtin_amdgcn_readfirstlane(s.est);
      s.iter = __builtin_amdgcn_readfirstlane(s.iter);
    }
    double x;
#if AIRICE_ROOTS_STAMP == 2
    const unsigned long long tn0 = dbg_clock();
    const bool more = s.next_point(M, x);
    const unsigned long long tn1 = dbg_clock() + (unsigned long long)(0.0 * x);
    rs_next += (int)(tn1 - tn0);
    if (!more) break;
#else
    if (!s.next_point(M, x)) break;
#endif
    // the single evaluation site: MinimizeforLaunchAngle (.cc:873-917)
    DBG_EXEC(4);
    double thd_air, thd_ice;
    const int ph = s.phase;
    if constexpr (WAVE) {
      if (have_next) {
        thd_air = next_air;
        thd_ice = next_ice;
        have_next = false;
      } else {
        // the point the next trip evaluates when this one is f(lo) (then f(hi)) or the first guard
        // (then always the second: PH_G1 -> PH_G2)
        const bool pair = ph == PH_FLO || ph == PH_G1;
        const double xb = ph == PH_FLO ? s.hi : s.x2 + s.dlt();
#if AIRICE_SCALAR_STAMP
        const unsigned long long e0 = dbg_clock();
        t_pre += (int)(e0 - tq) + (int)(0.0 * x);
#endif
        eval_thd_wave(M, I, s.q, x, pair ? xb : x, tab, thd_air, thd_ice, next_air, next_ice);
#if AIRICE_SCALAR_STAMP
        // debug: evaluation ticks in n_inside (the wave form does not count midpoints)
        tq = dbg_clock();
        s.n_inside += (int)(tq - e0) + (int)(0.0 * (thd_air + thd_ice));
#endif
        have_next = pair;
      }
    } else {
#if AIRICE_ROOTS_STAMP == 2
      const unsigned long long te0 = dbg_clock() + (unsigned long long)(0.0 * x);
      eval_thd(M, I, s.q, x, tab, thd_air, thd_ice);
      rs_eval += (int)(dbg_clock() + (unsigned long long)(0.0 * (thd_air + thd_ice)) - te0);
#else
      eval_thd(M, I, s.q, x, tab, thd_air, thd_ice);
#endif
    }
#if AIRICE_ROOTS_STAMP == 2
    const unsigned long long tu0 = dbg_clock() + (unsigned long long)(0.0 * (thd_air + thd_ice));
    s.template update<!WAVE>(M, x, thd_air, thd_ice);
    rs_upd += (int)(dbg_clock() + (unsigned long long)(0.0 * (s.lo + s.hi + s.x2)) - tu0);
#else
    s.template update<!WAVE>(M, x, thd_air, thd_ice);
#endif
    // f(hi) is not wanted after all when f(lo) was not finite
    if (WAVE && ph == PH_FLO && s.phase != PH_FHI) have_next = false;
#if AIRICE_SCALAR_STAMP
    if constexpr (WAVE) {
      const unsigned long long te = dbg_clock();
      t_post += (int)(te - tq) + (int)(0.0 * (s.lo + s.hi + s.x2));
      tq = te;
    }
#endif
  }
#if AIRICE_SCALAR_STAMP
  SolveResult sr{s.root(), s.status, s.n_eval, s.est, s.n_inside};
  sr.t_setup = t_setup;
  sr.t_lean = s.t_lean;
  sr.t_pre = t_pre;
  sr.t_post = t_post;
  return sr;
#else
  SolveResult sr{s.root(), s.status, s.n_eval, s.est, s.n_inside};
#if AIRICE_ROOTS_STAMP == 3
  for (int i = 0; i < 6; ++i) sr.tb[i] = s.tb[i];
#endif
#if AIRICE_ROOTS_STAMP == 2
  sr.t_next = rs_next;
  sr.t_eval = rs_eval;
  sr.t_upd = rs_upd;
  sr.t_pre = (int)(rs_l0 - ts_entry);
  sr.t_begin = (int)(ts_begun - ts_entry);
#endif
  return sr;
#endif
}

struct Solved {
  double launch, thd_air, t_air, geo_air, inc, thd_ice, t_ice, geo_ice, ant;
  double ice_n;  // Getnz_air(IceLayerHeight) after the Rx-in-air shift
  int status;
};

// Outputs at the root (GetAirPropagationPar + GetIcePropagationPar, .cc:1524-1566).
__host__ __device__ __forceinline__ Solved evaluate_root(const DevMedium& M, const IceConsts& I,
                                                const Geometry& g, double x, int status,
                                                const double* tab) {
  Solved S;
  S.status = status;
  S.launch = x;
  const AirPath P = make_air_path(M, g.H, g.ice);
  S.ice_n = P.iceair.n;
  S.thd_air = 0.0;
  S.t_air = 0.0;
  S.geo_air = 0.0;
  S.inc = __builtin_nan("");
  double L0 = __builtin_nan("");
  if (P.top < P.bot) {
    S.status |= AIRICE_SOLVE_NO_AIR_LAYER;
  } else {
    const double v2 = first_layer_v2(M, P.tx.n, P.rtop.n, x);
    L0 = P.rtop.n * v2;
    const double A2 = M.A_air * M.A_air;
    const RayL RL = ray_L(A2, L0);
    // the layer loop top -> bot as in air_thd: Tx layer, layers strictly between (uniform ends),
    // ice layer; same summation order
    auto add = [&](const Segment& sg) {
      S.thd_air += sg.thd;
      S.t_air += sg.t;
      S.geo_air += sg.geo;
    };
    add(segment(P.tx, P.rtop, M.A_air, A2, RL, true, tab));
#pragma unroll
    for (int il = kMaxLayers - 2; il >= 1; --il)
      if (il < P.top && il > P.bot) add(segment(M.start[il], M.stop[il], M.A_air, A2, RL, true, tab));
    if (P.top > P.bot) add(segment(start_endpoint(M, P.bot), P.iceair, M.A_air, A2, RL, true, tab));
    // receive angle of the last layer: asin(v2) for the first layer, asin(L0/n(Stop)) below
    S.inc = k_asin(P.top == P.bot ? v2 : L0 / P.iceair.n) * M.r2d;
  }
  S.thd_ice = 0.0;
  S.t_ice = 0.0;
  S.geo_ice = 0.0;
  S.ant = 0.0;
  if (g.depth < 0) {
    const Endpoint rx = ice_endpoint(M, g.depth_pos);
    const double A2i = M.A_ice * M.A_ice;
    const RayL RL = ray_L(A2i, L0);
    const Segment sg = segment(I.ice0, rx, M.A_ice, A2i, RL, false, tab);
    S.thd_ice = sg.thd;
    S.ant = k_asin(L0 / rx.n) * M.r2d;
    S.t_ice = sg.t;
    S.geo_ice = sg.geo;
  }
  return S;
}

// evaluate_root for one-query calls (scalar_solve_kernel; every lane holds the same query and
// root): the four air segments -- Tx layer, layers 2 and 1, the ice layer -- on lanes 0-3 at once
// (as eval_thd_wave), the segment in the ice beside them on every lane, then every lane forms the
// sums from the lanes' values in evaluate_root's order.  The same bits with about a quarter of
// its dependent chain.
__device__ __forceinline__ Solved evaluate_root_wave(const DevMedium& M, const IceConsts& I,
                                                     const Geometry& g, double x, int status,
                                                     const double* tab) {
  const int lane = (int)(threadIdx.x & 63);
  // branch-free (selects on wave-uniform conditions): one straight block, so the angle chains
  // (asin of the incidence and of the receive angle) overlap the segments
  Solved S;
  S.launch = x;
  const AirPath P = make_air_path(M, g.H, g.ice);
  S.ice_n = P.iceair.n;
  const bool air = !(P.top < P.bot);
  S.status = air ? status : (status | AIRICE_SOLVE_NO_AIR_LAYER);
  const double v2 = first_layer_v2(M, P.tx.n, P.rtop.n, x);
  const double L0 = air ? P.rtop.n * v2 : __builtin_nan("");
  const double inc = k_asin(P.top == P.bot ? v2 : L0 / P.iceair.n) * M.r2d;
  const Endpoint rx = ice_endpoint(M, g.depth_pos);
  const double ant = k_asin(L0 / rx.n) * M.r2d;
  // lanes 0-3: the air segments, with the kernel-uniform A as evaluate_root has it (the same
  // instruction forms, hence also the same NaN bits on rays without a solution)
  const double A2 = M.A_air * M.A_air;
  const RayL RL = ray_L(A2, L0);
  Endpoint T = P.tx, R = P.rtop;  // lane 0 (and the lanes past 3, whose value is unused)
  T = pick(lane == 1, M.start[2], T);
  R = pick(lane == 1, M.stop[2], R);
  T = pick(lane == 2, M.start[1], T);
  R = pick(lane == 2, M.stop[1], R);
  T = pick(lane == 3, start_endpoint(M, P.bot), T);
  R = pick(lane == 3, P.iceair, R);
  const Segment sg = segment(T, R, M.A_air, A2, RL, true, tab);
  // the segment in the ice on every lane, beside the air segments (used when g.depth < 0)
  const double A2i = M.A_ice * M.A_ice;
  const RayL RLi = ray_L(A2i, L0);
  const Segment si = segment(I.ice0, rx, M.A_ice, A2i, RLi, false, tab);
  auto from = [&](int l) { return Segment{__shfl(sg.thd, l), __shfl(sg.t, l), __shfl(sg.geo, l)}; };
  const Segment s0 = from(0), s1 = from(1), s2 = from(2), s3 = from(3);
  double thd = 0.0, t = 0.0, geo = 0.0;
  auto add = [&](bool c, const Segment& a) {
    thd = c ? thd + a.thd : thd;
    t = c ? t + a.t : t;
    geo = c ? geo + a.geo : geo;
  };
  add(air, s0);
  add(air && 2 < P.top && 2 > P.bot, s1);
  add(air && 1 < P.top && 1 > P.bot, s2);
  add(air && P.top > P.bot, s3);
  S.thd_air = thd;
  S.t_air = t;
  S.geo_air = geo;
  S.inc = air ? inc : __builtin_nan("");
  const bool in_ice = g.depth < 0;
  S.thd_ice = in_ice ? si.thd : 0.0;
  S.t_ice = in_ice ? si.t : 0.0;
  S.geo_ice = in_ice ? si.geo : 0.0;
  S.ant = in_ice ? ant : 0.0;
  return S;
}

// The root found by the one-query kernel, handed to its stage-2 body directly (WAVE) instead of
// through the parked output slots.
struct WaveRoot {
  double root;
  int status;
  Geometry g;  // the query, as load_query gave it to the root finder
};

__host__ __device__ __forceinline__ double straight_angle(const DevMedium& M, double H, double D, double ice,
                                                 double depth) {
  double thR = 0;
  if (depth < 0) thR = 180 - (atan(D / (H - ice - depth)) * M.r2d);
  if (depth >= 0) thR = 180 - (atan(D / (H - (ice + depth))) * M.r2d);
  return thR;
}

// Query sources.  IN_M: metres, uniform ice (Air2IceRayTracing batch); IN_CM: centimetres
// (GetHorizontalDistanceToIntersectionPoint, .cc:947-950); IN_TRACE: per-query ice, metres
// (TraceIceToAir).
// IN_CM100: the table lookup's minimizer fallback (.cc:1419), which hands the already-cm
// source/distance/depth over multiplied by 100 again (and the ice height, already in m, x100).
enum { IN_M = 0, IN_CM = 1, IN_TRACE = 2, IN_CM100 = 3 };

struct QueryArgs {
  const double* a;    // IN_M: txh    IN_CM(100): src_cm   IN_TRACE: depth
  const double* b;    //       dist               dist_cm            ice
  const double* c;    //       depth              depth_cm           txh
  const double* d;    //       thR (opt.)         -                  dist
  double ice;         // uniform ice height (m) or ice_cm for IN_CM(100)
  long long n;
  const uint8_t* mask;  // IN_CM100: only lanes with AIRICE_LOOKUP_FALLBACK set
};

// inl: a one-query call whose inputs arrived in the kernel arguments (Signal::in, the same values
// as Q's arrays hold), read from there instead of from host memory.
template <int IN>
__host__ __device__ __forceinline__ Geometry load_query(const DevMedium& M, const QueryArgs& Q, long long k,
                                               double& thR, const Signal* inl = nullptr) {
  const double qa = inl ? inl->in[0] : Q.a[k];
  const double qb = inl ? inl->in[1] : Q.b[k];
  const double qc = inl ? inl->in[2] : Q.c[k];
  double H, D, ice, dep;
  if (IN == IN_M) {
    H = qa;
    D = qb;
    dep = qc;
    ice = Q.ice;
    thR = Q.d != nullptr ? (inl ? inl->in[3] : Q.d[k]) : straight_angle(M, H, D, ice, dep);
  } else if (IN == IN_CM) {
    H = qa / 100;
    D = qb / 100;
    ice = Q.ice / 100;
    dep = qc / 100;
    thR = straight_angle(M, H, D, ice, dep);
  } else if (IN == IN_CM100) {
    H = (qa * 100) / 100;
    D = (qb * 100) / 100;
    ice = Q.ice / 100;
    dep = (qc * 100) / 100;
    thR = straight_angle(M, H, D, ice, dep);
  } else {
    dep = qa;
    ice = qb;
    H = qc;
    D = inl ? inl->in[3] : Q.d[k];
    thR = straight_angle(M, H, D, ice, dep);
  }
  return shift(H, D, ice, dep);
}

// A query's raw inputs as the grouping pass stores them in sorted order (group_scatter_kernel):
// {a, b, c, d} of QueryArgs at the query's index (d: IN_M's thR when given, IN_TRACE's dist).
struct QueryRec {
  double a, b, c, d;
};

// load_query<IN> on a stored record: the same arithmetic on the same values.
template <int IN>
__device__ __forceinline__ Geometry load_rec(const DevMedium& M, const QueryArgs& Q,
                                             const QueryRec& r, double& thR) {
  Signal s{};
  s.n_in = 4;
  s.in[0] = r.a;
  s.in[1] = r.b;
  s.in[2] = r.c;
  s.in[3] = r.d;
  return load_query<IN>(M, Q, 0, thR, &s);
}

// Stage 1's (root, status) of a grouped batch, in sorted order; stage 2 finds query k's record
// at inv[k].  rec == nullptr: the parked output slots (Park) hold them.
struct SortedPark {
  const double2* rec;
  const int* inv;
};

// Where stage 1 parks (root, status) for stage 2.
struct Park {
  double* root;
  double* status;
  long long stride;
  int exact;  // 1: evaluate every bisection midpoint (AIRICE_BISECT_EXACT, validation only)
  int* stats; // debug (AIRICE_SOLVE_STATS): per query {evaluations, secant search, midpoints}
};

// Debug/validation switch: AIRICE_BISECT_EXACT=1 makes the root finder evaluate f at every
// bisection midpoint instead of predicting the signs the guards determine (same roots).
static inline int bisect_exact() {
  const char* e = getenv("AIRICE_BISECT_EXACT");
  return (e != nullptr && e[0] == '1') ? 1 : 0;
}

// Lanes of a wave run until its slowest query is solved, and the number of f-evaluations
// follows the geometry (near-horizontal queries probe and need more secant steps).  So the block
// first groups its queries by straight-line angle (a 24-bucket counting sort in LDS) and each
// lane then solves the query of its slot: waves hold similar queries (per-wave maximum 10.3 ->
// ~8.2 evaluations on cfg3, 0.52 -> 0.45 ms per 1e6 solves).  Every query is still solved on its
// own and written by its index.
// (round 5, six alternating A/B rounds of the cfg3 solve call, same outputs: 16 buckets median
// 0.2377 ms, 24 buckets 0.2351, 64 buckets 0.2362; 8 angle classes x the layers spanned 0.241)
constexpr int kSortBuckets = 24;
// 1024 queries per block: larger groups sort better, and a 16-wave block runs at 4 waves/SIMD
// (128 VGPRs) -- measured faster than 256 (3 waves, no spills), 512 and 768; and (round 5) than
// 512- and 256-thread blocks that each sort the whole 1,024-query chunk (a deterministic ballot
// sort) and solve their half / quarter of it: the same waves at a finer dispatch grain, 0.263 /
// 0.307 against 0.244 ms per call (the duplicated keying costs more than the block tail saves).
constexpr int kRootsBlock = 1024;
constexpr int kRootsWaves = 4;  // 127 VGPRs: 4 waves/SIMD (5 and 6 spill and run slower)
// batch-wide grouping: trace (IN_TRACE) batches of at least kGroupMin queries are sorted across
// the whole batch and solved in kSortedBlock-thread blocks (roots_sorted_kernel; group_min_batch:
// the other sources stay block-local, AIRICE_GROUP_MIN in the environment overrides it)
constexpr long long kGroupMin = 65536;

// Stage 2 of the lookup fallback with the root handed over in registers (lookup_kernel):
// defined below.
__host__ __device__ __forceinline__ void fallback_out_direct(const DevMedium& M, const IceConsts& I,
                                                    const QueryArgs& Q, double* __restrict__ out,
                                                    size_t ld, uint8_t* __restrict__ ok,
                                                    long long k, const double* tab,
                                                    const Geometry& g, double root, int status);

constexpr int kGroupAngles = 8;   // straight-line-angle classes (16 measured +0.4 %)
// the classes within each angle class are the number of air layers the path spans (0-3+): a wave
// then runs only the middle-layer segments its own queries have
constexpr int kGroupHeights = 4;
// The sort key is roots_kernel's straight-line-angle bucket, b = floor((thR - 90) * B / 90) with
// thR = 180 - atan(x) deg, x = D / (H - ice - depth), evaluated without the atan: b >= j exactly
// when x <= tan(90 deg * (1 - j / B)), so b counts the host-computed thresholds x lies below.
// (The key only orders the work; results do not depend on it.)
struct GroupKey {
  double t[kGroupAngles];  // t[j - 1] = tan(90 deg * (1 - j / B)), j = 1 .. B-1
};

template <int IN>
__device__ __forceinline__ int query_bucket(const DevMedium& M, const QueryArgs& Q, long long k,
                                            const GroupKey& K) {
  if (IN == IN_CM100 && !(Q.mask[k] & AIRICE_LOOKUP_FALLBACK)) return -1;  // not a fallback lane
  double thR_unused;
  const Geometry g = load_query<IN>(M, Q, k, thR_unused);
  const double den = g.H - g.ice - g.depth;
  int b = 0;
  if (!(den > 0)) {
    b = den < 0 ? kGroupAngles - 1 : 0;  // thR > 180 (clamped) / 90 or NaN
  } else {
#pragma unroll
    for (int j = 0; j < kGroupAngles - 1; ++j) b += (g.D <= K.t[j] * den) ? 1 : 0;
  }
  const int span = top_layer(M, g.H) - bottom_layer(M, g.ice);
  return b * kGroupHeights + (span < 0 ? 0 : (span > 3 ? 3 : span));
}

// (the table lookup's fallback solves only its flagged lanes: lookup_kernel, not this)
constexpr bool solves_every_lane(int in) { return in != IN_CM100; }

template <int IN>
__global__ __launch_bounds__(kRootsBlock, kRootsWaves) void roots_kernel(DevMedium M, IceConsts I,
                                                                         QueryArgs Q, Park park) {
  static_assert(solves_every_lane(IN), "IN_CM100 lanes are masked: use lookup_kernel");
#if AIRICE_ROOTS_STAMP
  const unsigned long long st0 = __builtin_amdgcn_s_memtime();
#endif
  __shared__ int s_count[kSortBuckets + 1];
  __shared__ int s_slot[kRootsBlock];
  __shared__ double s_q[6][kRootsBlock];  // the sorted queries' geometry and straight-line angle
  const long long k0 = (long long)blockIdx.x * kRootsBlock;
  const long long kt = k0 + threadIdx.x;
  // the log table in LDS (one 16-byte entry per thread), as in table_kernel: every evaluation's
  // log ratios read it instead of global memory
  __shared__ __align__(16) double s_logtab[1 << kLogTableBits][2];
  for (unsigned t = threadIdx.x; t < (1u << kLogTableBits); t += kRootsBlock) {
    s_logtab[t][0] = kLogTable[t][0];
    s_logtab[t][1] = kLogTable[t][1];
  }
  if (threadIdx.x <= kSortBuckets) s_count[threadIdx.x] = 0;
  // the batch's ice end, once per block (IN_TRACE queries carry their own ice height)
  __shared__ IceAirPre s_ice;
  constexpr bool kIcePre = IN != IN_TRACE;
  if (kIcePre && threadIdx.x == 0) {
    const double ice = IN == IN_M ? Q.ice : Q.ice / 100;  // load_query's ice before the shift
    s_ice.x = ice;
    s_ice.bot = bottom_layer(M, ice);
    s_ice.s = air_slim(M, ice, s_ice.n);
  }
  // bucket of this lane's own query (unused lanes last); its inputs are read while the log table
  // is staged
  int bucket = kSortBuckets;
  Geometry g0{};
  double thR0 = 0.0;
  if (kt < Q.n) {
    g0 = load_query<IN>(M, Q, kt, thR0);
    const double b = (thR0 - 90.0) * (kSortBuckets / 90.0);
    bucket = (b >= 0.0 && b < kSortBuckets) ? (int)b : ((b >= kSortBuckets) ? kSortBuckets - 1 : 0);
  }
  __syncthreads();
  const int rank = atomicAdd(&s_count[bucket], 1);
  __syncthreads();
  // the first slot of the lane's bucket: the sizes of the buckets below it (independent LDS reads)
  int slot = rank;
#pragma unroll
  for (int b = 0; b < kSortBuckets; ++b) slot += b < bucket ? s_count[b] : 0;
  // the query moves to its slot through LDS: index, geometry and angle (no second global read)
  s_slot[slot] = threadIdx.x;
  s_q[0][slot] = g0.H;
  s_q[1][slot] = g0.D;
  s_q[2][slot] = g0.ice;
  s_q[3][slot] = g0.depth;
  s_q[4][slot] = g0.depth_pos;
  s_q[5][slot] = thR0;
  __syncthreads();
  const long long k = k0 + s_slot[threadIdx.x];
  if (k >= Q.n) return;
#if AIRICE_ROOTS_STAMP
  const unsigned long long st1 = __builtin_amdgcn_s_memtime() + (unsigned long long)(k & 0);
#endif
  Geometry g;
  g.H = s_q[0][threadIdx.x];
  g.D = s_q[1][threadIdx.x];
  g.ice = s_q[2][threadIdx.x];
  g.depth = s_q[3][threadIdx.x];
  g.depth_pos = s_q[4][threadIdx.x];
  const double thR = s_q[5][threadIdx.x];
#if AIRICE_ROOTS_STAMP
  const unsigned long long st2 =
      __builtin_amdgcn_s_memtime() + (unsigned long long)(0.0 * (thR + g.H + g.D + g.depth + g.ice));
#endif
  const SolveResult r = solve_root(M, I, g, thR, park.exact != 0, &s_logtab[0][0],
                                   kIcePre ? &s_ice : nullptr);
  st_agent(park.root + k * park.stride, r.root);
  st_agent(park.status + k * park.stride, (double)r.status);
#if AIRICE_ROOTS_STAMP
  const unsigned long long st3 = __builtin_amdgcn_s_memtime() + (unsigned long long)(0.0 * r.root);
  if (park.stats != nullptr) {
#if AIRICE_ROOTS_STAMP == 3
    park.stats[8 * k] = (int)(unsigned)st0 + 0 * (int)(st1 - st0);
    park.stats[8 * k + 1] = (int)(st3 - st2);
    for (int i = 0; i < 6; ++i) park.stats[8 * k + 2 + i] = r.tb[i];
#elif AIRICE_ROOTS_STAMP == 2
    // the search split: next_point, the evaluations and the rest (update, loop control)
    park.stats[7 * k] = (int)(unsigned)st0 + 0 * (int)(st1 - st0);
    park.stats[7 * k + 1] = (int)(st3 - st2);
    park.stats[7 * k + 2] = r.t_eval;
    park.stats[7 * k + 3] = r.t_next;
    park.stats[7 * k + 4] = r.t_upd;
    park.stats[7 * k + 5] = r.t_pre;
    park.stats[7 * k + 6] = r.t_begin;
#else
    park.stats[4 * k] = (int)(unsigned)st0;
    park.stats[4 * k + 1] = (int)(st1 - st0);
    park.stats[4 * k + 2] = (int)(st2 - st0);
    park.stats[4 * k + 3] = (int)(st3 - st0);
#endif
  }
#else
  if (park.stats != nullptr) {
    park.stats[3 * k] = r.n_eval;
    park.stats[3 * k + 1] = r.n_est;
    park.stats[3 * k + 2] = r.n_inside;
  }
#endif
}

// ---------------------------------------------------------------------------
// Batch-wide grouping (large batches).  roots_kernel above sorts inside each 1024-query block, so
// a CU -- which holds one such block at 128 VGPRs -- waits for the block's slowest wave before
// the next block can start.  Here the whole batch is first grouped by the same straight-line
// angle key (counting sort: keys + histogram, then a scatter), and roots_sorted_kernel solves the
// queries in that order in small blocks that the CU replaces independently.  Each query is still
// solved on its own and written by its index: results are identical either way.
// ---------------------------------------------------------------------------
constexpr int kGroupBuckets = kGroupAngles * kGroupHeights;
constexpr int kGroupItems = 2;  // queries per thread in the sort passes
constexpr int kGroupThreads = 1024;  // threads per block of the sort passes
constexpr int kGroupChunk = kGroupThreads * kGroupItems;  // queries per block and round
constexpr int kGroupBlocks = 512;                     // blocks of the sort passes (at most)
constexpr int kSortedBlock = 256;

// Pass 1: the key of every query and each block's bucket counts, bucket-major:
// cnt[b * nblocks + block] (no global atomics: thousands of blocks adding into a few counters
// serialise on them).  Both passes use at most kGroupBlocks blocks of kGroupThreads threads
// (8 waves/SIMD when the batch fills them), each block taking `rounds` chunks in turn.
template <int IN>
__global__ __launch_bounds__(kGroupThreads) void group_count_kernel(DevMedium M, QueryArgs Q,
                                                                    GroupKey K, int rounds,
                                                                    int8_t* __restrict__ key,
                                                                    int* __restrict__ cnt) {
  __shared__ int s_c[kGroupBuckets];
  if (threadIdx.x < kGroupBuckets) s_c[threadIdx.x] = 0;
  __syncthreads();
  for (int rr = 0; rr < rounds; ++rr) {
    const long long k0 = ((long long)blockIdx.x * rounds + rr) * kGroupChunk + threadIdx.x;
#pragma unroll
    for (int i = 0; i < kGroupItems; ++i) {
      const long long k = k0 + i * kGroupThreads;
      if (k < Q.n) {
        const int b = query_bucket<IN>(M, Q, k, K);
        key[k] = (int8_t)b;
        if (b >= 0) atomicAdd(&s_c[b], 1);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < kGroupBuckets) cnt[threadIdx.x * gridDim.x + blockIdx.x] = s_c[threadIdx.x];
}

// Pass 2: perm[position] = query index, positions grouped by bucket.  Each block first derives
// its own first position per bucket from all blocks' counts (bucket b's earlier buckets in full,
// plus bucket b of the blocks before it): kLanesPerBucket lanes per bucket sum strided slices of
// cnt[] and a tree in LDS adds them up, so no separate scan pass is needed.  A block's queries
// of one bucket take consecutive positions.
static_assert(kGroupThreads % kGroupBuckets == 0, "lanes per bucket");
constexpr int kLanesPerBucket = kGroupThreads / kGroupBuckets;
static_assert((kLanesPerBucket & (kLanesPerBucket - 1)) == 0, "power-of-two lanes per bucket");
template <int IN>
__global__ __launch_bounds__(kGroupThreads) void group_scatter_kernel(
    QueryArgs Q, const int8_t* __restrict__ key, long long n, int rounds,
    const int* __restrict__ cnt, int* __restrict__ grouped, int* __restrict__ inv,
    QueryRec* __restrict__ recs) {
  __shared__ int s_tot[kGroupBuckets][kLanesPerBucket], s_pre[kGroupBuckets][kLanesPerBucket];
  __shared__ int s_base[kGroupBuckets];
  const int nb = gridDim.x, blk = blockIdx.x;
  // this block's first-round keys, loaded before the prefix work so their latency overlaps it
  int b0[kGroupItems];
  const long long kb = (long long)blk * rounds * kGroupChunk + threadIdx.x;
#pragma unroll
  for (int i = 0; i < kGroupItems; ++i)
    b0[i] = kb + i * kGroupThreads < n ? (int)key[kb + i * kGroupThreads] : -1;
  const int bb = threadIdx.x / kLanesPerBucket, l = threadIdx.x % kLanesPerBucket;
  {
    const int* c = cnt + (long long)bb * nb;
    int tot = 0, pre = 0;
#pragma unroll 4
    for (int j = l; j < nb; j += kLanesPerBucket) {
      const int v = c[j];
      tot += v;
      pre += j < blk ? v : 0;
    }
    s_tot[bb][l] = tot;
    s_pre[bb][l] = pre;
  }
  __syncthreads();
#pragma unroll
  for (int h = kLanesPerBucket / 2; h > 0; h >>= 1) {
    if (l < h) {
      s_tot[bb][l] += s_tot[bb][l + h];
      s_pre[bb][l] += s_pre[bb][l + h];
    }
    __syncthreads();
  }
  if (threadIdx.x < kGroupBuckets) {
    int base = s_pre[threadIdx.x][0];
    for (int b = 0; b < (int)threadIdx.x; ++b) base += s_tot[b][0];
    s_base[threadIdx.x] = base;
    if (blk == 0 && threadIdx.x == kGroupBuckets - 1)  // number of queries with a bucket
      *grouped = base + s_tot[kGroupBuckets - 1][0];
  }
  __syncthreads();
  for (int rr = 0; rr < rounds; ++rr) {
    const long long k0 = ((long long)blk * rounds + rr) * kGroupChunk + threadIdx.x;
#pragma unroll
    for (int i = 0; i < kGroupItems; ++i) {
      const long long k = k0 + i * kGroupThreads;
      const int b = rr == 0 ? b0[i] : (k < n ? (int)key[k] : -1);
      if (b >= 0) {
        // the query's inputs move to its sorted position (one 32-byte record), so the root finder
        // reads them contiguously; inv[k] tells stage 2 where the query's result is parked
        const int pos = atomicAdd(&s_base[b], 1);
        const bool has_d = IN == IN_TRACE || (IN == IN_M && Q.d != nullptr);
        recs[pos] = QueryRec{Q.a[k], Q.b[k], Q.c[k], has_d ? Q.d[k] : 0.0};
        inv[k] = pos;
      }
    }
  }
}

template <int IN>
__global__ __launch_bounds__(kSortedBlock, kRootsWaves) void roots_sorted_kernel(
    DevMedium M, IceConsts I, QueryArgs Q, Park park, const QueryRec* __restrict__ recs,
    double2* __restrict__ sorted_park, const int* __restrict__ grouped) {
  __shared__ __align__(16) double s_logtab[1 << kLogTableBits][2];
  for (int t = threadIdx.x; t < (1 << kLogTableBits); t += kSortedBlock) {
    s_logtab[t][0] = kLogTable[t][0];
    s_logtab[t][1] = kLogTable[t][1];
  }
  __syncthreads();
  const long long ks = (long long)blockIdx.x * kSortedBlock + threadIdx.x;
  static_assert(solves_every_lane(IN), "IN_CM100 lanes are masked: use lookup_kernel");
  if (ks >= *grouped) return;  // past the queries with a bucket
  DBG_EXEC(12);
  double thR;
  const Geometry g = load_rec<IN>(M, Q, recs[ks], thR);
  const SolveResult r = solve_root(M, I, g, thR, park.exact != 0, &s_logtab[0][0]);
  sorted_park[ks] = make_double2(r.root, (double)r.status);
#if AIRICE_SORTED_STATS
  // debug build: evaluation counts by sorted position, i.e. in the order the waves run them
  if (park.stats != nullptr) {
    park.stats[3 * ks] = r.n_eval;
    park.stats[3 * ks + 1] = r.n_est;
    park.stats[3 * ks + 2] = r.n_inside;
  }
#endif
}

// Stage 1's result of query k for stage 2.
__host__ __device__ __forceinline__ void parked(const SortedPark& sp, const double* root_slot,
                                       const double* status_slot, long long k, double& x, int& st) {
  if (sp.rec != nullptr) {
    const double2 p = sp.rec[sp.inv[k]];
    x = p.x;
    st = (int)p.y;
  } else {
    x = *root_slot;
    st = (int)*status_slot;
  }
}

__host__ __device__ __forceinline__ bool check_solution(double thd, double D) {
  // CheckSolution (.cc:978-983, AirIceRayTracing.cc:916-921)
  bool good = false;
  if ((fabs(thd - D) / D < 0.01 && D <= 100) || (fabs(thd - D) < 1 && D > 100)) good = true;
  if (thd < 0) good = false;
  return good;
}

// The stage-2 kernels read the log table from LDS like the solve.
__device__ __forceinline__ void stage_log_table(double (*s)[2]) {
  for (unsigned t = threadIdx.x; t < (1u << kLogTableBits); t += kBlock) {
    s[t][0] = kLogTable[t][0];
    s[t][1] = kLogTable[t][1];
  }
  __syncthreads();
}

// Stage 2 of Air2IceRayTracing: dummy[0..16] (MultiRay, .cc:1597-1614) or dummy[0..14]
// (pythonwrapper, AirIceRayTracing.cc:1070-1084), SoA with stride ld.
// Stage-2 bodies (one query k, parked root in its output slots), shared by the batch out kernels
// and the one-query fused kernel (scalar_solve_kernel).
// WAVE (one-query kernel): every lane runs the body with the root in wr; evaluate_root_wave
// spreads the evaluation over the wave and lane 0 writes the outputs.
// Stage-2 output stores (non-temporal stores measured no faster)
// (agent-scope stores: cfg3 solve call 0.2359-0.2370 -> 0.2352-0.2358 ms with the parked roots
// stored the same way, same outputs; the lookup's non-temporal stores stay: 101.7 against 102.4 us)
__host__ __device__ __forceinline__ void put_out(double* p, double v) { st_agent(p, v); }

template <int VARIANT, bool WAVE = false>
__host__ __device__ __forceinline__ void solve_out_body(const DevMedium& M, const IceConsts& I,
                                               const QueryArgs& Q, double* __restrict__ out,
                                               size_t ld, uint8_t* __restrict__ status,
                                               long long k, const double* tab,
                                               WaveRoot wr = WaveRoot{0.0, 0},
                                               SortedPark sp = SortedPark{nullptr, nullptr}) {
  double thR;
  const Geometry g = WAVE ? wr.g : load_query<IN_M>(M, Q, k, thR);
  double x = wr.root;
  int st = wr.status;
  if (!WAVE) parked(sp, out + 10 * ld + k, out + 0 * ld + k, k, x, st);
  Solved S;
  if constexpr (WAVE) {
    S = evaluate_root_wave(M, I, g, x, st, tab);
    if (threadIdx.x != 0) return;
  } else {
    S = evaluate_root(M, I, g, x, st, tab);
  }
  const double thd = S.thd_ice + S.thd_air;
  const double tt = S.t_ice + S.t_air;
  put_out(out + 0 * ld + k, g.H);
  put_out(out + 1 * ld + k, thd);
  put_out(out + 2 * ld + k, S.thd_air);
  put_out(out + 3 * ld + k, S.thd_ice);
  put_out(out + 4 * ld + k, tt * kSpeedC);
  put_out(out + 5 * ld + k, S.t_ice * kSpeedC);
  put_out(out + 6 * ld + k, S.t_air * kSpeedC);
  put_out(out + 7 * ld + k, tt);
  put_out(out + 8 * ld + k, S.t_ice);
  put_out(out + 9 * ld + k, S.t_air);
  put_out(out + 10 * ld + k, S.launch);
  if (VARIANT == AIRICE_VARIANT_MULTIRAY) {
    double tS, tP;
    fresnel_from_sine(S.ice_n, I.ice0.n, S.ice_n / I.ice0.n, sin_start(S.inc * M.d2r), tS, tP);
    put_out(out + 11 * ld + k, S.ant);
    put_out(out + 12 * ld + k, tS);
    put_out(out + 13 * ld + k, tP);
    put_out(out + 14 * ld + k, S.geo_air);
    put_out(out + 15 * ld + k, S.geo_ice);
    put_out(out + 16 * ld + k, S.inc);
  } else {
    put_out(out + 11 * ld + k, k_asin((S.ice_n / I.ice0.n) * sin_start(S.inc * M.d2r)) * M.r2d);
    put_out(out + 12 * ld + k, S.ant);
    put_out(out + 13 * ld + k, S.geo_air);
    put_out(out + 14 * ld + k, S.geo_ice);
  }
  if (status != nullptr) status[k] = (uint8_t)S.status;
}

// occupancy of the stage-2 kernel: the compiler's choice (104 VGPRs, 4 waves/SIMD; held to 5-6
// waves it takes 80 VGPRs and runs within noise, at 8 it spills and runs slower: round 6)
template <int VARIANT>
__global__ __launch_bounds__(kBlock, kOutWaves) void solve_out_kernel(DevMedium M, IceConsts I, QueryArgs Q,
                                                           double* __restrict__ out, size_t ld,
                                                           uint8_t* __restrict__ status,
                                                           SortedPark sp) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  __shared__ __align__(16) double s_logtab[1 << kLogTableBits][2];
  stage_log_table(s_logtab);
  if (k >= Q.n) return;
  solve_out_body<VARIANT>(M, I, Q, out, ld, status, k, &s_logtab[0][0], WaveRoot{0.0, 0}, sp);
}

// Stage 2 of GetHorizontalDistanceToIntersectionPoint (.cc:945-989): 9 outputs (cm, rad) + bool.
template <bool WAVE = false>
__host__ __device__ __forceinline__ void hdtip_out_body(const DevMedium& M, const IceConsts& I,
                                               const QueryArgs& Q, double* __restrict__ out,
                                               size_t ld, uint8_t* __restrict__ ok, long long k,
                                               const double* tab, WaveRoot wr = WaveRoot{0.0, 0},
                                               SortedPark sp = SortedPark{nullptr, nullptr}) {
  double thR;
  const Geometry g = WAVE ? wr.g : load_query<IN_CM>(M, Q, k, thR);
  double x = wr.root;
  int st = wr.status;
  if (!WAVE) parked(sp, out + 4 * ld + k, out + 0 * ld + k, k, x, st);
  Solved S;
  if constexpr (WAVE) {
    S = evaluate_root_wave(M, I, g, x, st, tab);
    if (threadIdx.x != 0) return;
  } else {
    S = evaluate_root(M, I, g, x, st, tab);
  }
  const double thd = S.thd_ice + S.thd_air;
  double tS, tP;
  fresnel_from_sine(S.ice_n, I.ice0.n, S.ice_n / I.ice0.n, sin_start(S.inc * M.d2r), tS, tP);
  out[0 * ld + k] = (S.t_ice * kSpeedC) * 100;
  out[1 * ld + k] = (S.t_air * kSpeedC) * 100;
  out[2 * ld + k] = S.geo_ice * 100;
  out[3 * ld + k] = S.geo_air * 100;
  out[4 * ld + k] = S.launch * M.d2r;
  out[5 * ld + k] = S.thd_air * 100;
  out[6 * ld + k] = tS;
  out[7 * ld + k] = tP;
  out[8 * ld + k] = S.ant * M.d2r;
  ok[k] = check_solution(thd, g.D) ? 1 : 0;
}

__global__ __launch_bounds__(kBlock, kOutWaves) void hdtip_out_kernel(DevMedium M, IceConsts I, QueryArgs Q,
                                                           double* __restrict__ out, size_t ld,
                                                           uint8_t* __restrict__ ok, SortedPark sp) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  __shared__ __align__(16) double s_logtab[1 << kLogTableBits][2];
  stage_log_table(s_logtab);
  if (k >= Q.n) return;
  hdtip_out_body(M, I, Q, out, ld, ok, k, &s_logtab[0][0], WaveRoot{0.0, 0}, sp);
}

// Stage 2 of the table lookup's minimizer fallback (.cc:1417-1456): the reference passes its
// own output references to GetHorizontalDistanceToIntersectionPoint in the order
// (geoIce, geoAir, optIce, optAir, ...), so the optical and geometric slots trade places;
// `ok` arrives holding the lookup's checks and is completed with CheckSolBool and
// launchAngle < 0, then the four zeroed slots of .cc:1451-1456.
// DIRECT (lane form): the query and its root arrive in wr (the fused fallback pass) instead of
// being reloaded and read back from the parked slots.
template <bool WAVE = false, bool DIRECT = false>
__host__ __device__ __forceinline__ void lookup_fallback_out_body(const DevMedium& M, const IceConsts& I,
                                                         const QueryArgs& Q,
                                                         double* __restrict__ out, size_t ld,
                                                         uint8_t* __restrict__ ok, long long k,
                                                         const double* tab,
                                                         WaveRoot wr = WaveRoot{0.0, 0}) {
  if (!(Q.mask[k] & AIRICE_LOOKUP_FALLBACK)) return;
  double thR;
  const Geometry g = (WAVE || DIRECT) ? wr.g : load_query<IN_CM100>(M, Q, k, thR);
  const double x = (WAVE || DIRECT) ? wr.root : out[4 * ld + k];
  const int st = (WAVE || DIRECT) ? wr.status : (int)out[0 * ld + k];
  Solved S;
  if constexpr (WAVE) {
    S = evaluate_root_wave(M, I, g, x, st, tab);
    if (threadIdx.x != 0) return;
  } else {
    S = evaluate_root(M, I, g, x, st, tab);
  }
  const double thd = S.thd_ice + S.thd_air;
  double tS, tP;
  fresnel_from_sine(S.ice_n, I.ice0.n, S.ice_n / I.ice0.n, sin_start(S.inc * M.d2r), tS, tP);
  const double launch = S.launch * M.d2r;
  const bool good = ok[k] != 0 && check_solution(thd, g.D) && !(launch < 0);
  out[0 * ld + k] = good ? S.geo_ice * 100 : 0.0;
  out[1 * ld + k] = good ? S.geo_air * 100 : 0.0;
  out[2 * ld + k] = (S.t_ice * kSpeedC) * 100;
  out[3 * ld + k] = (S.t_air * kSpeedC) * 100;
  out[4 * ld + k] = good ? launch : 0.0;
  out[5 * ld + k] = good ? S.thd_air * 100 : 0.0;
  out[6 * ld + k] = tS;
  out[7 * ld + k] = tP;
  out[8 * ld + k] = S.ant * M.d2r;
  ok[k] = good ? 1 : 0;
}

__host__ __device__ __forceinline__ void fallback_out_direct(const DevMedium& M, const IceConsts& I,
                                                    const QueryArgs& Q, double* __restrict__ out,
                                                    size_t ld, uint8_t* __restrict__ ok,
                                                    long long k, const double* tab,
                                                    const Geometry& g, double root, int status) {
  lookup_fallback_out_body<false, true>(M, I, Q, out, ld, ok, k, tab, WaveRoot{root, status, g});
}

// Stage 2 of the pythonwrapper TraceIceToAir (TraceIceToAir.C:5-73), rows of 10.
template <bool WAVE = false>
__host__ __device__ __forceinline__ void trace_out_body(const DevMedium& M, const IceConsts& I,
                                               const QueryArgs& Q, double* __restrict__ out10,
                                               long long k, const double* tab,
                                               WaveRoot wr = WaveRoot{0.0, 0},
                                               SortedPark sp = SortedPark{nullptr, nullptr}) {
  double thR;
  const Geometry g = WAVE ? wr.g : load_query<IN_TRACE>(M, Q, k, thR);
  double* o = out10 + 10 * k;
  double x = wr.root;
  int st = wr.status;
  if (!WAVE) parked(sp, o + 5, o + 9, k, x, st);
  Solved S;
  if constexpr (WAVE) {
    S = evaluate_root_wave(M, I, g, x, st, tab);
    if (threadIdx.x != 0) return;
  } else {
    S = evaluate_root(M, I, g, x, st, tab);
  }
  const double thd = S.thd_ice + S.thd_air;
  const double aoi = k_asin((S.ice_n / I.ice0.n) * sin_start(S.inc * M.d2r)) * M.r2d;
  if (check_solution(thd, g.D)) {
    // swap(launch, received); received = 180 - received (TraceIceToAir.C:33-34)
    o[0] = g.H;
    o[1] = g.D;
    o[2] = S.geo_ice;
    o[3] = S.geo_air;
    o[4] = S.ant;
    o[5] = 180 - S.launch;
    o[6] = S.thd_air;
    o[7] = aoi;
    o[8] = 0;
    o[9] = 0;
  } else {
#pragma unroll
    for (int c = 0; c < 10; ++c) o[c] = -1000;
  }
}

__global__ __launch_bounds__(kBlock, kTraceOutWaves) void trace_out_kernel(DevMedium M, IceConsts I, QueryArgs Q,
                                                           double* __restrict__ out10,
                                                           SortedPark sp) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  __shared__ __align__(16) double s_logtab[1 << kLogTableBits][2];
  stage_log_table(s_logtab);
  if (k >= Q.n) return;
  trace_out_body(M, I, Q, out10, k, &s_logtab[0][0], WaveRoot{0.0, 0}, sp);
}

// One query, both stages in one launch (the scalar C++ / ctypes entry points): one wave finds the
// root with the evaluation spread over its lanes, then runs the stage-2 body of the entry point
// (OUT) with its evaluation spread the same way.  Bit-identical to the two batch kernels.
enum { OUT_SOLVE_MR = 0, OUT_SOLVE_PY = 1, OUT_HDTIP = 2, OUT_FALLBACK = 3, OUT_TRACE = 4 };
template <int IN, int OUT>
// (of park only the exact flag is used: the root goes to the stage-2 body directly)
__global__ __launch_bounds__(64) void scalar_solve_kernel(DevMedium M, IceConsts I, QueryArgs Q,
                                                          Park park, double* out, size_t ld,
                                                          uint8_t* flag, Signal sig) {
  prefetch_kernargs<sizeof(DevMedium) + sizeof(IceConsts)>();
#if AIRICE_SCALAR_STAMP
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
#endif
  // one wave and a handful of logarithms per evaluation: the log table is read from global
  // memory (L1 / L2 after the first call) instead of being staged in LDS first
  const double* tab = &kLogTable[0][0];
  if (IN == IN_CM100 && !(Q.mask[0] & AIRICE_LOOKUP_FALLBACK)) {
    if (threadIdx.x == 0) signal_done(sig);
    return;
  }
  double thR;
#if AIRICE_SCALAR_STAMP
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
#endif
  const Geometry g = load_query<IN>(M, Q, 0, thR, 
                                    sig.n_in >= ((IN == IN_TRACE || (IN == IN_M && Q.d != nullptr)) ? 4 : 3)
                                        ? &sig
                                        : nullptr);
  const SolveResult r = solve_root<true>(M, I, g, thR, park.exact != 0, tab);
#if AIRICE_SCALAR_STAMP
  const unsigned long long c2 = __builtin_amdgcn_s_memtime();
#endif
  // every lane runs the stage-2 body (its evaluation spread over the wave); lane 0 writes
  const WaveRoot wr{r.root, r.status, g};
  if (OUT == OUT_SOLVE_MR)
    solve_out_body<AIRICE_VARIANT_MULTIRAY, true>(M, I, Q, out, ld, flag, 0, tab, wr);
  if (OUT == OUT_SOLVE_PY)
    solve_out_body<AIRICE_VARIANT_PYWRAPPER, true>(M, I, Q, out, ld, flag, 0, tab, wr);
  if (OUT == OUT_HDTIP) hdtip_out_body<true>(M, I, Q, out, ld, flag, 0, tab, wr);
  if (OUT == OUT_FALLBACK) lookup_fallback_out_body<true>(M, I, Q, out, ld, flag, 0, tab, wr);
  if (OUT == OUT_TRACE) trace_out_body<true>(M, I, Q, out, 0, tab, wr);
  if (threadIdx.x != 0) return;
#if AIRICE_SCALAR_STAMP
  const unsigned long long c3 = __builtin_amdgcn_s_memtime(), w3 = __builtin_amdgcn_s_memrealtime();
  out[17 * ld] = (double)(c1 - c0);
  out[18 * ld] = (double)(c2 - c1);
  out[19 * ld] = (double)(c3 - c2);
  out[20 * ld] = (double)(c3 - c0);
  out[21 * ld] = (double)(w3 - w0);
  out[22 * ld] = (double)r.n_eval;
  out[23 * ld] = (double)r.n_inside;
  out[24 * ld] = (double)r.t_setup;
  out[25 * ld] = (double)r.t_lean;
  out[26 * ld] = (double)r.t_pre;
  out[27 * ld] = (double)r.t_post;
#endif
  signal_done(sig);
}

// One query of a minimizer entry point on the host (AIRICE_SCALAR_HOST, the default of the
// one-query C++ / ctypes drop-ins): the root finder and the entry point's stage-2 body compiled
// for the CPU from the same source as the batch kernels (the host's correctly rounded sqrt and
// quotients in place of the device iterations).  The root is the GSL bisection's, decided by the
// signs of f at its midpoints, so it is the device's; the outputs at it agree to an ulp or so.
// Q: the query at index 0 (host pointers); park: where stage 1 parks (root, status) for the body,
// as the launcher of the batch path sets it.
template <int IN, int OUT>
static void solve_one_host_t(const DevMedium& M, const IceConsts& I, const QueryArgs& Q,
                             const Park& park, double* out, size_t ld, uint8_t* flag) {
  const double* tab = &kLogTable[0][0];
  if (IN == IN_CM100 && !(Q.mask[0] & AIRICE_LOOKUP_FALLBACK)) return;
  double thR;
  const Geometry g = load_query<IN>(M, Q, 0, thR);
  const SolveResult r = solve_root<false>(M, I, g, thR, park.exact != 0, tab);
  if constexpr (OUT == OUT_FALLBACK) {
    fallback_out_direct(M, I, Q, out, ld, flag, 0, tab, g, r.root, r.status);
  } else {
    park.root[0] = r.root;
    park.status[0] = (double)r.status;
    if constexpr (OUT == OUT_SOLVE_MR)
      solve_out_body<AIRICE_VARIANT_MULTIRAY>(M, I, Q, out, ld, flag, 0, tab);
    if constexpr (OUT == OUT_SOLVE_PY)
      solve_out_body<AIRICE_VARIANT_PYWRAPPER>(M, I, Q, out, ld, flag, 0, tab);
    if constexpr (OUT == OUT_HDTIP) hdtip_out_body(M, I, Q, out, ld, flag, 0, tab);
    if constexpr (OUT == OUT_TRACE) trace_out_body(M, I, Q, out, 0, tab);
  }
}

// Air2IceRayTracing, one query (in: txh, dist, depth [, straight angle]): out17 / out15 with
// ld = 1 (as launch_solve parks and writes), status bits.
int solve_host_one(const DevMedium& M, const IceConsts& I, int variant, const double* in,
                   bool has_thr, double* out, uint8_t* status) {
  const QueryArgs Q{in, in + 1, in + 2, has_thr ? in + 3 : nullptr, I.ice_h, 1};
  const Park park{out + 10, out, 1, bisect_exact(), nullptr};
  if (variant == AIRICE_VARIANT_PYWRAPPER)
    solve_one_host_t<IN_M, OUT_SOLVE_PY>(M, I, Q, park, out, 1, status);
  else
    solve_one_host_t<IN_M, OUT_SOLVE_MR>(M, I, Q, park, out, 1, status);
  return AIRICE_OK;
}

// GetHorizontalDistanceToIntersectionPoint, one query (in: src, dist, depth in cm).
int hdtip_host_one(const DevMedium& M, const IceConsts& I, double ice_cm, const double* in,
                   double* out9, uint8_t* ok) {
  const QueryArgs Q{in, in + 1, in + 2, nullptr, ice_cm, 1};
  const Park park{out9 + 4, out9, 1, bisect_exact(), nullptr};
  solve_one_host_t<IN_CM, OUT_HDTIP>(M, I, Q, park, out9, 1, ok);
  return AIRICE_OK;
}

// TraceIceToAir, one query (in: depth, ice, txh, dist).
int trace_host_one(const DevMedium& M, const IceConsts& I, const double* in, double* out10) {
  const QueryArgs Q{in, in + 1, in + 2, in + 3, 0.0, 1};
  const Park park{out10 + 5, out10 + 9, 10, bisect_exact(), nullptr};
  solve_one_host_t<IN_TRACE, OUT_TRACE>(M, I, Q, park, out10, 0, nullptr);
  return AIRICE_OK;
}

// The table lookup's minimizer fallback for one flagged query (in: src, dist, depth in cm; ok and
// flags as the lookup left them).
int lookup_fallback_host_one(const DevMedium& M, const IceConsts& I, double ice_cm,
                             const double* in, double* out9, uint8_t* ok, const uint8_t* flags) {
  const double ice_arg = (ice_cm / 100) * 100;  // as launch_lookup_fallback (.cc:1309, 1419)
  const QueryArgs Q{in, in + 1, in + 2, nullptr, ice_arg, 1, flags};
  const Park park{out9 + 4, out9, 1, bisect_exact(), nullptr};
  solve_one_host_t<IN_CM100, OUT_FALLBACK>(M, I, Q, park, out9, 1, ok);
  return AIRICE_OK;
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
static inline unsigned grid_for(long long n) { return (unsigned)((n + kBlock - 1) / kBlock); }
static inline int launch_ok() { return hipGetLastError() == hipSuccess ? AIRICE_OK : AIRICE_EHIP; }

static inline dim3 roots_grid(size_t n) {
  return dim3((unsigned)((n + kRootsBlock - 1) / kRootsBlock));
}

// Stream-ordered scratch for the grouping passes: a library-owned pool per device whose release
// threshold keeps freed blocks for reuse (the default pool returns them at every synchronisation,
// and re-growing it made each launch wait on the host).
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t st) {
  static std::mutex mu;
  static std::vector<hipMemPool_t> pools;
  int dev = 0;
  if (hipError_t e = hipGetDevice(&dev)) return e;
  hipMemPool_t pool = nullptr;
  {
    std::lock_guard<std::mutex> lock(mu);
    if ((int)pools.size() <= dev) pools.resize(dev + 1, nullptr);
    if (pools[dev] == nullptr) {
      hipMemPoolProps props{};
      props.allocType = hipMemAllocationTypePinned;
      props.location.type = hipMemLocationTypeDevice;
      props.location.id = dev;
      if (hipError_t e = hipMemPoolCreate(&pools[dev], &props)) return e;
      uint64_t keep = UINT64_MAX;
      (void)hipMemPoolSetAttribute(pools[dev], hipMemPoolAttrReleaseThreshold, &keep);
    }
    pool = pools[dev];
  }
  return hipMallocFromPoolAsync(p, bytes, pool, st);
}

static const GroupKey& group_thresholds() {
  static const GroupKey K = [] {
    GroupKey k{};
    for (int j = 1; j < kGroupAngles; ++j)
      k.t[j - 1] = tan(M_PI / 2 * (1.0 - (double)j / kGroupAngles));
    return k;
  }();
  return K;
}

// Measured with the slope-placed guards (round 4): cfg3 (IN_M, 1e6) 0.241 ms per call
// block-local against 0.276 ms grouped -- four to five evaluations per query leave the 1,024-query
// blocks' angle sort as good as the batch-wide one, and the grouping passes and the stage-2 gather
// cost more -- while cfg5 (IN_TRACE, 1e7, Tx up to 20 km, per-query ice) takes 2.23 ms grouped
// against 2.53 block-local.  So the batch-wide grouping is the default of the trace source only;
// AIRICE_GROUP_MIN overrides it for every source (0: never group).
size_t group_min_batch(int in) {
  static const char* env = getenv("AIRICE_GROUP_MIN");
  static const long long v = env ? atoll(env) : -1;
  if (v >= 0) return (size_t)v;
  return in == IN_TRACE ? (size_t)kGroupMin : 0;
}

// Stage 1 of every minimizer launch: roots_kernel (block-local grouping) for small batches and
// debug statistics, the batch-wide grouping otherwise (stream-ordered scratch, scratch_alloc).
// A grouped launch returns the sorted parking (sp) its stage-2 kernel reads, and the scratch
// block (ws) to release after that kernel (RootsScratch).
template <int IN>
static int launch_roots(const DevMedium& M, const IceConsts& I, const QueryArgs& Q,
                        const Park& park, size_t n, hipStream_t st, SortedPark& sp, void*& ws) {
  static_assert(solves_every_lane(IN), "IN_CM100 lanes are masked: use launch_lookup_fallback");
  sp = SortedPark{nullptr, nullptr};
  ws = nullptr;
  const size_t group_min = group_min_batch(IN);
  if (group_min == 0 || n < group_min ||
      (park.stats != nullptr && !AIRICE_SORTED_STATS) || n >= (1ull << 31)) {
    ktimer_begin(KT_ROOTS, st);
    count_launch(LC_ROOTS);
    hipLaunchKernelGGL((roots_kernel<IN>), roots_grid(n), dim3(kRootsBlock), 0, st, M, I, Q, park);
    ktimer_end(KT_ROOTS, st);
    return launch_ok();
  }
  const GroupKey& thresholds = group_thresholds();
  // at most kGroupBlocks blocks in the two passes (each scatter block reads every block's
  // counts); larger batches give each block several chunks
  const size_t chunks = (n + kGroupChunk - 1) / kGroupChunk;
  const int rounds = (int)((chunks + kGroupBlocks - 1) / kGroupBlocks);
  const unsigned nb = (unsigned)((chunks + rounds - 1) / rounds);
  const size_t m = (size_t)kGroupBuckets * nb;
  // scratch: sorted query records (32 B), sorted (root, status) (16 B), inv (4 B) and key (1 B)
  // per query, then the bucket counts and the grouped count
  const size_t ws_bytes = (sizeof(QueryRec) + sizeof(double2) + sizeof(int) + 1) * n +
                          sizeof(int) * (m + 1);
  if (scratch_alloc(&ws, ws_bytes, st) != hipSuccess) return AIRICE_EHIP;
  QueryRec* recs = static_cast<QueryRec*>(ws);
  double2* sorted = reinterpret_cast<double2*>(recs + n);
  int* inv = reinterpret_cast<int*>(sorted + n);
  int* cnt = inv + n;
  int* grouped = cnt + m;
  int8_t* key = reinterpret_cast<int8_t*>(grouped + 1);
  ktimer_begin(KT_GROUP, st);
  hipLaunchKernelGGL(group_count_kernel<IN>, dim3(nb), dim3(kGroupThreads), 0, st, M, Q,
                     thresholds, rounds, key, cnt);
  hipLaunchKernelGGL(group_scatter_kernel<IN>, dim3(nb), dim3(kGroupThreads), 0, st, Q, key,
                     (long long)n, rounds, cnt, grouped, inv, recs);
  ktimer_end(KT_GROUP, st);
  const unsigned sorted_blocks = (unsigned)((n + kSortedBlock - 1) / kSortedBlock);
  ktimer_begin(KT_ROOTS, st);
  count_launch(LC_ROOTS);
  hipLaunchKernelGGL(roots_sorted_kernel<IN>, dim3(sorted_blocks), dim3(kSortedBlock), 0, st, M, I,
                     Q, park, recs, sorted, grouped);
  ktimer_end(KT_ROOTS, st);
  sp = SortedPark{sorted, inv};
  return launch_ok();
}

// A grouped launch's scratch block, released stream-ordered after its stage-2 kernel
// (release()), or on any early return by the destructor.
struct RootsScratch {
  void* ws = nullptr;
  hipStream_t st;
  explicit RootsScratch(hipStream_t s) : st(s) {}
  RootsScratch(const RootsScratch&) = delete;
  RootsScratch& operator=(const RootsScratch&) = delete;
  ~RootsScratch() {
    if (ws != nullptr) (void)hipFreeAsync(ws, st);
  }
  int release() {
    void* p = ws;
    ws = nullptr;
    if (p != nullptr && hipFreeAsync(p, st) != hipSuccess) return AIRICE_EHIP;
    return AIRICE_OK;
  }
};

// Per-grid device caches of the table launch: the row constants of every Tx-height row
// (RowConst, 104 B; rowconst_kernel) and the start-angle sine of every grid column (8 B;
// angle_sines_kernel).  Both are O(rows + columns) work that every block of a launch would
// otherwise redo for the rows and columns it touches.
//
// Life of an entry (GridCache::get):
//  - the FIRST launch that needs a key records the key only and forms its rows / sines in the
//    kernel (rc / vs = nullptr): a grid built once -- one table per antenna, RunMultiRayCode.C's
//    pattern -- pays no fill kernel, no allocation and no synchronisation;
//  - the SECOND launch with the key allocates the buffer, enqueues the fill kernel on its own
//    stream ahead of its table kernel (stream order makes the buffer complete for it) and records
//    an event behind the fill; no host synchronisation;
//  - later launches use the buffer: on the filling stream directly, on another stream once the
//    event has completed (hipEventQuery) or behind a hipStreamWaitEvent on it;
//  - a launch being captured into a graph uses an entry only if its fill is already known to be
//    complete, and pins it: a pinned buffer is never evicted (its address lives in the graph's
//    kernel arguments).  Otherwise the captured launch forms its rows / sines in the kernel.  No
//    allocation, query or fill happens under capture.
// A buffer is written once and never overwritten.  At most kCacheSets unpinned entries per device;
// the least recently used is freed with hipFree, which waits for the kernels still reading it.
// The caller holds grid_cache_mutex() from the lookup until its launches are enqueued, so no other
// thread can evict a buffer in between; a multi-antenna launch touches at most kMaxAntennas
// (< kCacheSets) entries, so its own are never the least recently used.
static std::mutex& grid_cache_mutex() {
  static std::mutex mu;
  return mu;
}
// A stream that is being captured into a graph (no allocation, query or synchronisation then).
static bool stream_capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}
constexpr size_t kCacheSets = 64;
static_assert(kMaxAntennas < (int)kCacheSets, "a multi-antenna launch never evicts its own entries");

class GridCache {
 public:
  // fill(buffer, stream): enqueue the kernel that writes the whole buffer.  fill_first: fill at
  // the key's first use already (large launches, where forming the values in the kernel costs
  // more than the fill kernel).
  template <class Fill>
  int get(const std::vector<unsigned char>& key, size_t bytes, hipStream_t st, Fill fill,
          bool fill_first, const void** out) {
    *out = nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return AIRICE_EHIP;
    if (per_dev_.size() <= (size_t)dev) per_dev_.resize(dev + 1);
    Dev& D = per_dev_[dev];
    Entry* c = nullptr;
    for (Entry& e : D.entries)
      if (e.key == key) c = &e;
    if (stream_capturing(st)) {
      if (c != nullptr && c->dev != nullptr && c->ready) {
        c->pinned = true;
        c->used = ++D.tick;
        *out = c->dev;
      }
      return AIRICE_OK;  // otherwise the captured kernel forms the values itself
    }
    if (c == nullptr) {  // first use: remember the key, the kernel forms the values
      if (int rc = make_room(D)) return rc;
      Entry e;
      e.key = key;
      e.used = ++D.tick;
      D.entries.push_back(std::move(e));
      if (!fill_first) return AIRICE_OK;
      c = &D.entries.back();
    }
    c->used = ++D.tick;
    if (c->dev == nullptr) {  // second use: fill, stream-ordered ahead of this launch
      void* p = nullptr;
      if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) return AIRICE_EHIP;
      fill(p, st);
      hipEvent_t ev = nullptr;
      if (hipGetLastError() != hipSuccess ||
          hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
          hipEventRecord(ev, st) != hipSuccess) {
        if (ev != nullptr) (void)hipEventDestroy(ev);
        (void)hipFree(p);
        return AIRICE_EHIP;
      }
      c->dev = p;
      c->ev = ev;
      c->origin = st;
      *out = p;
      return AIRICE_OK;
    }
    if (!c->ready) {
      const hipError_t q = hipEventQuery(c->ev);
      if (q == hipSuccess) {
        c->ready = true;
      } else if (q != hipErrorNotReady) {
        return AIRICE_EHIP;
      } else if (st != c->origin && hipStreamWaitEvent(st, c->ev, 0) != hipSuccess) {
        return AIRICE_EHIP;
      }
    }
    *out = c->dev;
    return AIRICE_OK;
  }

  // entries of the current device (tests: airice_table_cache_stats)
  void stats(int* keys, int* filled, int* pinned) {
    int dev = 0;
    *keys = *filled = *pinned = 0;
    if (hipGetDevice(&dev) != hipSuccess || per_dev_.size() <= (size_t)dev) return;
    for (const Entry& e : per_dev_[dev].entries) {
      ++*keys;
      *filled += e.dev != nullptr;
      *pinned += e.pinned;
    }
  }

 private:
  struct Entry {
    std::vector<unsigned char> key;
    void* dev = nullptr;        // nullptr: seen once, not filled
    hipEvent_t ev = nullptr;    // recorded behind the fill kernel
    hipStream_t origin = nullptr;
    bool ready = false;         // the fill is known complete
    bool pinned = false;        // handed to a captured launch: never evicted
    unsigned long long used = 0;
  };
  struct Dev {
    std::vector<Entry> entries;
    unsigned long long tick = 0;
  };
  // evict the least recently used unpinned entry when kCacheSets unpinned entries exist
  static int make_room(Dev& D) {
    size_t unpinned = 0, old = D.entries.size();
    for (size_t k = 0; k < D.entries.size(); ++k) {
      if (D.entries[k].pinned) continue;
      ++unpinned;
      if (old == D.entries.size() || D.entries[k].used < D.entries[old].used) old = k;
    }
    if (unpinned < kCacheSets) return AIRICE_OK;
    Entry& e = D.entries[old];
    if (e.dev != nullptr && hipFree(e.dev) != hipSuccess) return AIRICE_EHIP;
    if (e.ev != nullptr) (void)hipEventDestroy(e.ev);
    D.entries.erase(D.entries.begin() + (long)old);
    return AIRICE_OK;
  }
  std::vector<Dev> per_dev_;
};

static GridCache& row_cache() {
  static GridCache c;
  return c;
}
static GridCache& angle_cache() {
  static GridCache c;
  return c;
}

// The row constants of a grid.  row_const reads the medium, the heights and, of the ice constants,
// only the lowest air layer (bot) and the Tx-layer stop ends (topend): the key holds exactly those,
// so tables of one grid for antennas at different depths in the ice share one entry.
// Rays of a launch from which a grid's caches are filled at its first use: forming the rows and
// sines in the kernel costs ~2-5 ps per ray (cfg2: +2 us, 1.07x; cfg4 at 8.7e8 rays: +4.3 ms,
// 1.21x), the two fill kernels ~10-20 us.
constexpr long long kFillFirstRays = 1LL << 22;

static int row_consts_cached(const DevMedium& M, const IceConsts& I, const TableArgs& A,
                             hipStream_t st, bool fill_first, const RowConst** out) {
  const double gk[3] = {A.start_h, A.stop_h, A.step_h};
  std::vector<unsigned char> key(sizeof(M) + sizeof(I.bot) + sizeof(I.topend) + sizeof(gk) +
                                 sizeof(A.hsteps));
  unsigned char* kp = key.data();
  std::memcpy(kp, &M, sizeof(M));
  kp += sizeof(M);
  std::memcpy(kp, &I.bot, sizeof(I.bot));
  kp += sizeof(I.bot);
  std::memcpy(kp, I.topend, sizeof(I.topend));
  kp += sizeof(I.topend);
  std::memcpy(kp, gk, sizeof(gk));
  kp += sizeof(gk);
  std::memcpy(kp, &A.hsteps, sizeof(A.hsteps));
  auto fill = [&](void* p, hipStream_t s) {
    hipLaunchKernelGGL(rowconst_kernel, dim3((unsigned)((A.hsteps + 255) / 256)), dim3(256), 0, s,
                       M, I, A, static_cast<RowConst*>(p));
  };
  const void* p = nullptr;
  const int rc = row_cache().get(key, sizeof(RowConst) * (size_t)std::max(A.hsteps, 1), st, fill,
                                 fill_first, &p);
  *out = static_cast<const RowConst*>(p);
  return rc;
}

// The start-angle sines of an angle grid (the degree-to-radian factor and the angle grid).
static int angle_sines_cached(const DevMedium& M, const TableArgs& A, hipStream_t st,
                              bool fill_first, const double** out) {
  const double k5[5] = {M.d2r, A.start_a, A.stop_a, A.step_a, (double)A.asteps};
  std::vector<unsigned char> key(sizeof(k5));
  std::memcpy(key.data(), k5, sizeof(k5));
  auto fill = [&](void* p, hipStream_t s) {
    hipLaunchKernelGGL(angle_sines_kernel, dim3((unsigned)((A.asteps + 255) / 256)), dim3(256), 0,
                       s, M, A, static_cast<double*>(p));
  };
  const void* p = nullptr;
  const int rc = angle_cache().get(key, sizeof(double) * (size_t)std::max(A.asteps, 1), st, fill,
                                   fill_first, &p);
  *out = static_cast<const double*>(p);
  return rc;
}

#if AIRICE_SORTED_STATS
int debug_exec_counters(unsigned long long* out, int n, int reset) {
  if (n > 16) n = 16;
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg_exec), sizeof(unsigned long long) * n) != hipSuccess)
    return AIRICE_EHIP;
  if (reset) {
    static const unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_exec), z, sizeof(z)) != hipSuccess) return AIRICE_EHIP;
  }
  return AIRICE_OK;
}
#endif

void table_cache_stats(int out[6]) {
  std::lock_guard<std::mutex> lock(grid_cache_mutex());
  row_cache().stats(&out[0], &out[1], &out[2]);
  angle_cache().stats(&out[3], &out[4], &out[5]);
}

int launch_table(const DevMedium& M, const IceConsts& I, const airice_grid* g, int row_begin,
                 int row_count, float* d_table, double* d_full, size_t ld, hipStream_t st) {
  if (row_count <= 0 || g->angle_steps <= 0) return AIRICE_OK;
  TableArgs A;
  A.start_h = g->start_height;
  A.stop_h = g->stop_height;
  A.step_h = g->height_step;
  A.start_a = g->start_angle;
  A.stop_a = g->stop_angle;
  A.step_a = g->angle_step;
  A.hsteps = g->height_steps;
  A.asteps = g->angle_steps;
  A.in_ice = g->in_ice;
  A.ld = ld;
  A.inv_asteps = 1.0 / (double)g->angle_steps;
  // rows a 256-ray set can touch, for the LDS row constants
  A.rows_per_block = std::min(kTableBlock, (kTableBlock - 1) / g->angle_steps + 2);
  A.rc = nullptr;
  std::unique_lock<std::mutex> rs_lock(grid_cache_mutex());  // held until the launches are enqueued
  const bool fill_first = (long long)row_count * g->angle_steps >= kFillFirstRays;
  if (int rc = row_consts_cached(M, I, A, st, fill_first, &A.rc)) return rc;
  A.vs = nullptr;
  if (int rc = angle_sines_cached(M, A, st, fill_first, &A.vs)) return rc;
  static const char* trace_path = getenv("AIRICE_TABLE_TRACE");
  // ray indices are 32-bit inside a launch: grids of kMaxLaunchRays or more go in row slabs
  const int max_rows = (int)std::max<long long>(1, (kMaxLaunchRays - 2 * kTableBlock) / g->angle_steps);
  for (int done = 0; done < row_count;) {
    const int rows = std::min(max_rows, row_count - done);
    const size_t off = (size_t)done * (size_t)g->angle_steps;
    A.row0 = row_begin + done;
    A.n = rows * g->angle_steps;
    float* tab = d_table + off;
    double* full = d_full ? d_full + off : nullptr;
    done += rows;
    A.half = A.n;
    const size_t lds = sizeof(RowConst) * (size_t)A.rows_per_block;
    const unsigned blocks = (unsigned)((A.n + kTableBlock - 1) / kTableBlock);
    if (trace_path == nullptr) {
      ktimer_begin(KT_TABLE, st);
      count_launch(LC_TABLE);
      const bool sc1 = A.n < kAgentStoreRays;
      if (M.A_air == 1.0 && sc1)
        hipLaunchKernelGGL((table_kernel<false, true, true>), dim3(blocks), dim3(kTableBlock), lds,
                           st, M, I, A, tab, full, nullptr);
      else if (M.A_air == 1.0)
        hipLaunchKernelGGL((table_kernel<false, true, false>), dim3(blocks), dim3(kTableBlock), lds,
                           st, M, I, A, tab, full, nullptr);
      else if (sc1)
        hipLaunchKernelGGL((table_kernel<false, false, true>), dim3(blocks), dim3(kTableBlock), lds,
                           st, M, I, A, tab, full, nullptr);
      else
        hipLaunchKernelGGL((table_kernel<false, false, false>), dim3(blocks), dim3(kTableBlock), lds,
                           st, M, I, A, tab, full, nullptr);
      ktimer_end(KT_TABLE, st);
      if (hipGetLastError() != hipSuccess) return AIRICE_EHIP;
      continue;
    }
    // debug timeline (tools/wave_timeline.py): synchronous, one record per wave appended
    const long long nw = (long long)blocks * (kTableBlock / 64);
    WaveTrace* dtr = nullptr;
    if (hipMalloc(&dtr, sizeof(WaveTrace) * nw) != hipSuccess) return AIRICE_EHIP;
    hipLaunchKernelGGL((table_kernel<true, false, true>), dim3(blocks), dim3(kTableBlock), lds, st, M, I,
                       A, tab, full, dtr);
    std::vector<WaveTrace> h(nw);
    if (hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(h.data(), dtr, sizeof(WaveTrace) * nw, hipMemcpyDeviceToHost) != hipSuccess)
      return AIRICE_EHIP;
    (void)hipFree(dtr);
    if (FILE* f = fopen(trace_path, "ab")) {
      fwrite(h.data(), sizeof(WaveTrace), nw, f);
      fclose(f);
    }
  }
  return launch_ok();
}

// Several antennas' whole tables in one launch of table_multi_kernel.  Ih[a], grids[a]: antenna
// a's constants and grid (the rows it holds: grids[a].table_rows); tables[a] its output, column
// stride lds[a].  The per-antenna constants live in a device buffer per distinct set, kept for
// repeated launches of the same set (bench steps, repeated builds).
int launch_table_multi(const DevMedium& M, const IceConsts* Ih, const airice_grid* grids, int n,
                       float* const* tables, const size_t* lds, hipStream_t st) {
  if (n <= 0) return AIRICE_OK;
  if (n > kMaxAntennas) {
    set_error("at most %d antennas per multi-antenna launch", kMaxAntennas);
    return AIRICE_EINVAL;
  }
  std::vector<TableArgs> Ah(n);
  std::unique_lock<std::mutex> rs_lock(grid_cache_mutex());  // held until the launch is enqueued
  MultiMap map;
  std::memset(&map, 0, sizeof(map));
  map.n_ant = n;
  long long blocks = 0;
  const int rpb = [&] {
    int r = 2;
    for (int a = 0; a < n; ++a)
      r = std::max(r, std::min(kTableBlock, (kTableBlock - 1) / grids[a].angle_steps + 2));
    return r;
  }();
  for (int a = 0; a < n; ++a) {
    const airice_grid* g = &grids[a];
    TableArgs& A = Ah[a];
    std::memset(&A, 0, sizeof(A));
    A.start_h = g->start_height;
    A.stop_h = g->stop_height;
    A.step_h = g->height_step;
    A.start_a = g->start_angle;
    A.stop_a = g->stop_angle;
    A.step_a = g->angle_step;
    A.hsteps = g->height_steps;
    A.asteps = g->angle_steps;
    A.in_ice = g->in_ice;
    A.ld = lds[a];
    A.inv_asteps = 1.0 / (double)g->angle_steps;
    A.rows_per_block = rpb;
    A.row0 = 0;
    A.rc = nullptr;
    const bool fill_first = (long long)g->table_rows * g->angle_steps >= kFillFirstRays;
    if (int rc = row_consts_cached(M, Ih[a], A, st, fill_first, &A.rc)) return rc;
    A.vs = nullptr;
    if (int rc = angle_sines_cached(M, A, st, fill_first, &A.vs)) return rc;
    const long long rays = (long long)g->table_rows * g->angle_steps;
    if (rays >= kMaxLaunchRays - 2 * kTableBlock || lds[a] < (size_t)rays) {
      set_error("antenna %d: %lld rays (ld %zu) do not fit one multi-antenna launch", a, rays,
                lds[a]);
      return AIRICE_EINVAL;
    }
    A.n = (int)rays;
    A.half = A.n;
    map.begin[a] = (int)blocks;
    map.table[a] = tables[a];
    blocks += (rays + kTableBlock - 1) / kTableBlock;
  }
  map.begin[n] = (int)blocks;
  if (blocks == 0) return AIRICE_OK;
  // Device copies of the per-antenna constants, one immutable buffer per distinct constant set
  // (up to kConstSets per device, least recently used evicted).  A buffer is written once, by a
  // synchronous copy before any launch reads it, and never overwritten; eviction frees it with
  // hipFree, which waits for the kernels still reading it, on any stream.  The lock is held until
  // the launch is enqueued, so no other thread can evict the buffer in between.  Under graph
  // capture (no allocation or copy allowed) a launch needs its set to be resident already -- one
  // uncaptured launch of the same antenna set first -- and pins it: a pinned set is never evicted,
  // since the graph keeps its address.
  struct ConstSet {
    std::vector<unsigned char> host;
    void* dev = nullptr;
    unsigned long long used = 0;
    bool pinned = false;
  };
  constexpr size_t kConstSets = 8;
  static std::mutex mu;
  static std::vector<std::vector<ConstSet>> caches;
  static unsigned long long tick = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return AIRICE_EHIP;
  const size_t bytes_i = sizeof(IceConsts) * n, bytes = bytes_i + sizeof(TableArgs) * n;
  std::vector<unsigned char> packed(bytes);
  std::memcpy(packed.data(), Ih, bytes_i);
  std::memcpy(packed.data() + bytes_i, Ah.data(), sizeof(TableArgs) * n);
  std::lock_guard<std::mutex> lock(mu);
  if (caches.size() <= (size_t)dev) caches.resize(dev + 1);
  std::vector<ConstSet>& sets = caches[dev];
  ConstSet* c = nullptr;
  for (ConstSet& e : sets)
    if (e.host == packed) c = &e;
  const bool capturing = stream_capturing(st);
  if (c == nullptr && capturing) {
    set_error("multi-antenna table launch under graph capture: run one uncaptured launch of the "
              "same antenna set (twice: the grid caches fill on a grid's second launch) first");
    return AIRICE_EINVAL;
  }
  if (c == nullptr) {
    size_t unpinned = 0, old = sets.size();
    for (size_t k = 0; k < sets.size(); ++k) {
      if (sets[k].pinned) continue;
      ++unpinned;
      if (old == sets.size() || sets[k].used < sets[old].used) old = k;
    }
    if (unpinned >= kConstSets) {  // evict the least recently used unpinned set
      if (hipFree(sets[old].dev) != hipSuccess) return AIRICE_EHIP;
      sets.erase(sets.begin() + (long)old);
    }
    ConstSet e;
    if (hipMalloc(&e.dev, bytes) != hipSuccess) return AIRICE_EHIP;
    if (hipMemcpy(e.dev, packed.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(e.dev);
      return AIRICE_EHIP;
    }
    e.host = std::move(packed);
    sets.push_back(std::move(e));
    c = &sets.back();
  }
  c->used = ++tick;
  if (capturing) c->pinned = true;
  void* dconst = c->dev;
  const size_t lds_bytes = sizeof(RowConst) * (size_t)rpb;
  ktimer_begin(KT_TABLE, st);
  const bool sc1 = (long long)blocks * kTableBlock < kAgentStoreRays;
  auto multi = M.A_air == 1.0 ? (sc1 ? table_multi_kernel<true, true> : table_multi_kernel<true, false>)
                              : (sc1 ? table_multi_kernel<false, true> : table_multi_kernel<false, false>);
  count_launch(LC_TABLE);
  hipLaunchKernelGGL(multi, dim3((unsigned)blocks), dim3(kTableBlock),
                     lds_bytes, st, M, static_cast<const IceConsts*>(dconst),
                     reinterpret_cast<const TableArgs*>(static_cast<unsigned char*>(dconst) +
                                                        bytes_i),
                     map);
  ktimer_end(KT_TABLE, st);
  return launch_ok();
}

int launch_rays(const DevMedium& M, const IceConsts& I, const double* launch, const double* txh,
                int in_ice, size_t n, double* out, size_t ld, hipStream_t st) {
  if (n == 0) return AIRICE_OK;
  if (n == 1) {  // one ray: spread over a wave (ray_solution_wave)
    count_launch(LC_SCALAR_RAY);
    hipLaunchKernelGGL(scalar_ray_kernel, dim3(1), dim3(64), 0, st, M, I, launch, txh, in_ice, out,
                       ld, take_scalar_signal());
    return launch_ok();
  }
  count_launch(LC_RAYS);
  hipLaunchKernelGGL(rays_kernel, dim3(grid_for((long long)n)), dim3(kBlock), 0, st, M, I, launch,
                     txh, in_ice, (long long)n, out, ld, Signal{});
  return launch_ok();
}

// The one-query GetRayTracingSolutions on the host (airice_rays_host): ray_solution compiled for
// the CPU from the same source as rays_kernel -- the same operation sequence, with the host's
// correctly rounded sqrt and quotients in place of the device's v_rsq/v_rcp iterations (within
// ~1 ulp of them).  A one-ray launch costs a kernel dispatch and a completion wait (~8 us); the
// host ray takes ~1 us.
void rays_host(const DevMedium& M, const IceConsts& I, const double* launch, const double* txh,
               int in_ice, size_t n, double* out, size_t ld) {
  for (size_t k = 0; k < n; ++k) {
    double d[18];
    ray_solution(M, I, launch[k], txh[k], in_ice != 0, d);
    for (int c = 0; c < 18; ++c) out[c * ld + k] = d[c];
  }
}

int launch_solve(const DevMedium& M, const IceConsts& I, int variant, const double* txh,
                 const double* dist, const double* depth, const double* thr, size_t n,
                 double* out, size_t ld, uint8_t* status, hipStream_t st) {
  if (n == 0) return AIRICE_OK;
  const QueryArgs Q{txh, dist, depth, thr, I.ice_h, (long long)n};
  Park park{out + 10 * ld, out, 1, bisect_exact(), nullptr};
  static const char* stats_path = getenv("AIRICE_SOLVE_STATS");
  if (stats_path != nullptr && hipMalloc(&park.stats, sizeof(int) * kStatsInts * n) != hipSuccess)
    return AIRICE_EHIP;
  const dim3 grid(grid_for((long long)n)), block(kBlock);
  if (n == 1 && park.stats == nullptr) {
    const Signal sig = take_scalar_signal();
    count_launch(LC_SCALAR_SOLVE);
    if (variant == AIRICE_VARIANT_MULTIRAY)
      hipLaunchKernelGGL((scalar_solve_kernel<IN_M, OUT_SOLVE_MR>), dim3(1), dim3(64), 0, st, M, I,
                         Q, park, out, ld, status, sig);
    else
      hipLaunchKernelGGL((scalar_solve_kernel<IN_M, OUT_SOLVE_PY>), dim3(1), dim3(64), 0, st, M, I,
                         Q, park, out, ld, status, sig);
    return launch_ok();
  }
  SortedPark sp;
  RootsScratch scr(st);
  if (int rc = launch_roots<IN_M>(M, I, Q, park, n, st, sp, scr.ws)) return rc;
  if (park.stats != nullptr) {  // debug: append the per-query counts (synchronous)
    std::vector<int> h(kStatsInts * n);
    if (hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(h.data(), park.stats, sizeof(int) * kStatsInts * n, hipMemcpyDeviceToHost) != hipSuccess)
      return AIRICE_EHIP;
    (void)hipFree(park.stats);
    if (FILE* f = fopen(stats_path, "ab")) {
      fwrite(h.data(), sizeof(int), kStatsInts * n, f);
      fclose(f);
    }
  }
  ktimer_begin(KT_OUT, st);
  count_launch(LC_OUT);
  if (variant == AIRICE_VARIANT_MULTIRAY)
    hipLaunchKernelGGL(solve_out_kernel<AIRICE_VARIANT_MULTIRAY>, grid, block, 0, st, M, I, Q, out,
                       ld, status, sp);
  else
    hipLaunchKernelGGL(solve_out_kernel<AIRICE_VARIANT_PYWRAPPER>, grid, block, 0, st, M, I, Q,
                       out, ld, status, sp);
  ktimer_end(KT_OUT, st);
  const int rc = launch_ok();
  if (int rf = scr.release()) return rf;
  return rc;
}

int launch_hdtip(const DevMedium& M, const IceConsts& I, const double* src, const double* dist,
                 const double* depth, double ice_cm, size_t n, double* out, size_t ld,
                 uint8_t* ok, hipStream_t st) {
  if (n == 0) return AIRICE_OK;
  const QueryArgs Q{src, dist, depth, nullptr, ice_cm, (long long)n};
  const Park park{out + 4 * ld, out, 1, bisect_exact(), nullptr};
  const dim3 grid(grid_for((long long)n)), block(kBlock);
  if (n == 1) {
    count_launch(LC_SCALAR_SOLVE);
    hipLaunchKernelGGL((scalar_solve_kernel<IN_CM, OUT_HDTIP>), dim3(1), dim3(64), 0, st, M, I, Q,
                       park, out, ld, ok, take_scalar_signal());
    return launch_ok();
  }
  SortedPark sp;
  RootsScratch scr(st);
  if (int rc = launch_roots<IN_CM>(M, I, Q, park, n, st, sp, scr.ws)) return rc;
  ktimer_begin(KT_OUT, st);
  count_launch(LC_OUT);
  hipLaunchKernelGGL(hdtip_out_kernel, grid, block, 0, st, M, I, Q, out, ld, ok, sp);
  ktimer_end(KT_OUT, st);
  const int rc = launch_ok();
  if (int rf = scr.release()) return rf;
  return rc;
}

// The table lookup's minimizer fallback for one query (the one-query device call; a batch solves
// its fallback lanes inside lookup_kernel).
int launch_lookup_fallback(const DevMedium& M, const IceConsts& I, const double* src,
                           const double* dist, const double* depth, double ice_cm, size_t n,
                           double* out, size_t ld, uint8_t* ok, const uint8_t* flags,
                           hipStream_t st) {
  if (n == 0) return AIRICE_OK;
  // .cc:1309 turns IceLayerHeight into metres; .cc:1419 passes IceLayerHeight*100
  const double ice_arg = (ice_cm / 100) * 100;
  const QueryArgs Q{src, dist, depth, nullptr, ice_arg, (long long)n, flags};
  const Park park{out + 4 * ld, out, 1, bisect_exact(), nullptr};
  if (n != 1) {
    set_error("launch_lookup_fallback: one query (batches solve their fallback in lookup_kernel)");
    return AIRICE_EINVAL;
  }
  count_launch(LC_SCALAR_SOLVE);
  hipLaunchKernelGGL((scalar_solve_kernel<IN_CM100, OUT_FALLBACK>), dim3(1), dim3(64), 0, st, M,
                     I, Q, park, out, ld, ok, take_scalar_signal());
  return launch_ok();
}

// GetHorizontalDistanceToIntersectionPoint_Table (.cc:1305-1462) for a batch, one query per lane:
// lk_query (airice_lookup.hpp: row records, the THD window in LDS, pair records), and a lane whose
// query hits the one-sided case runs the reference's minimizer fallback (.cc:1418-1420: the root
// finder and its stage 2 with the root in registers) in place while the other waves go on with
// their lookups.  (Round 5: a separate fallback pass after the lookup launch -- 4,096-query
// chunks, flagged lanes listed in LDS -- waited for the whole launch and then for one solve's
// latency: 100.8-101.8 against 93.1-93.5 us per 1e6 random queries, same outputs.)
// 128 VGPRs (the root finder's cap, 4 waves/SIMD as the lookup alone at 97).
__global__ __launch_bounds__(kLkBlock, kRootsWaves) void lookup_kernel(
    LkTable T, DevMedium M, IceConsts I, QueryArgs Q, double* __restrict__ out, size_t ld,
    uint8_t* __restrict__ ok, uint8_t* __restrict__ flags, int exact) {
  const long long k = (long long)blockIdx.x * kLkBlock + threadIdx.x;
  if (k >= Q.n) return;
  if (T.ang != nullptr && *reinterpret_cast<const int*>(T.ang + (lk_angles_ok_offset(T.n, T.asteps) -
                                                                  lk_angles_offset(T.n, T.asteps))) == 0)
    T.ang = nullptr;
  __shared__ float s_win[kLkWindow][kLkBlock];
  int fl = 0;
  double o[9];
  bool good = false;
  const bool fb = lk_query(T, Q.a[k] / 100, Q.b[k] / 100, M.d2r, o, &good, fl, &s_win[0][threadIdx.x]);
  if (!fb) {
#pragma unroll
    for (int c = 0; c < 9; ++c) __builtin_nontemporal_store(o[c], out + c * ld + k);
  }
  ok[k] = good ? 1 : 0;
  flags[k] = (uint8_t)fl;
  if (fb) {
    double thR;
    const Geometry g = load_query<IN_CM100>(M, Q, k, thR);
    const SolveResult r = solve_root(M, I, g, thR, exact != 0, &kLogTable[0][0]);
    fallback_out_direct(M, I, Q, out, ld, ok, k, &kLogTable[0][0], g, r.root, r.status);
  }
}

int launch_lookup(const DevMedium& M, const IceConsts& I, const airice_lookup_table* t,
                  const double* src, const double* dist, const double* depth, double ice_cm,
                  size_t n, double* out, size_t ld, uint8_t* ok, uint8_t* flags, hipStream_t st) {
  if (n == 0) return AIRICE_OK;
  const LkTable T = lk_table(t);
  const double ice_arg = (ice_cm / 100) * 100;  // .cc:1309 in metres, .cc:1419 passes it x100
  const QueryArgs Q{src, dist, depth, nullptr, ice_arg, (long long)n, flags};
  const unsigned grid = (unsigned)((n + kLkBlock - 1) / kLkBlock);
  ktimer_begin(KT_LOOKUP, st);
  count_launch(LC_LOOKUP);
  hipLaunchKernelGGL(lookup_kernel, dim3(grid), dim3(kLkBlock), 0, st, T, M, I, Q, out, ld, ok,
                     flags, bisect_exact());
  ktimer_end(KT_LOOKUP, st);
  return launch_ok();
}

int launch_trace(const DevMedium& M, const IceConsts& I, const double* depth, const double* ice,
                 const double* txh, const double* dist, size_t n, double* out10, hipStream_t st) {
  if (n == 0) return AIRICE_OK;
  const QueryArgs Q{depth, ice, txh, dist, 0.0, (long long)n};
  const Park park{out10 + 5, out10 + 9, 10, bisect_exact(), nullptr};
  const dim3 grid(grid_for((long long)n)), block(kBlock);
  if (n == 1) {
    count_launch(LC_SCALAR_SOLVE);
    hipLaunchKernelGGL((scalar_solve_kernel<IN_TRACE, OUT_TRACE>), dim3(1), dim3(64), 0, st, M, I, Q,
                       park, out10, 0, nullptr, take_scalar_signal());
    return launch_ok();
  }
  SortedPark sp;
  RootsScratch scr(st);
  if (int rc = launch_roots<IN_TRACE>(M, I, Q, park, n, st, sp, scr.ws)) return rc;
  ktimer_begin(KT_OUT, st);
  count_launch(LC_OUT);
  hipLaunchKernelGGL(trace_out_kernel, grid, block, 0, st, M, I, Q, out10, sp);
  ktimer_end(KT_OUT, st);
  const int rc = launch_ok();
  if (int rf = scr.release()) return rf;
  return rc;
}

}  // namespace airice
