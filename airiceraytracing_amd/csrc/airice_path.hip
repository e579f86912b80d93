// airice_path.hip -- SingleRayAirIceRefraction (BASELINE cfg1) on gfx950: the forward trace of
// one launch angle with the RayTracingFunctions numerics, and the x(z) ray-path sampler that
// writes RayPathinAirnIce.txt (SingleRayAirIceRefraction.C:33-299).
//
//  single_ray_kernel : one lane.  Layer loop (.C:100-154: GetLayerHitPointPar for the Tx layer,
//                      the same L below, RayTracingFunctions.cc:399-514 / :349-369), the ice leg
//                      (GetIcePropagationPar, RayTracingFunctions.cc:661-679, positive depth),
//                      and the per-layer constants of the sampler: fDnfR at each layer's start
//                      height and the running x offset (LastRefracted_x, .C:285).
//  path_kernel       : one lane per path sample (1 m steps, ~17k for cfg1): its layer from
//                      the host-computed sample ranges, then one fDnfR (.C:254-258, 293-297).
//
// The sample count and each layer's start/stop heights are integer/height bookkeeping of the
// reference's own loops (.C:226-299) and are done on the host so the output can be sized; every
// refractive-index / ray quantity is computed on the device.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>

#include "airice.h"
#include "airice_internal.h"

namespace airice {

namespace {

constexpr double kSpeedC = 299792458.0;  // RayTracingFunctions.h spedc
constexpr int kPathBlock = 256;

struct PathPlan {
  int top;           // MaxLayers - SkipLayersAbove - 1 (first air layer of the trace, .C:100)
  int bot;           // SkipLayersBelow
  int nl;            // path layers = MaxLayers - SkipLayersAbove - SkipLayersBelow (.C:226)
  int pad_;
  double txh, ice, depth, launch;
  double start[kMaxLayers], stop[kMaxLayers];  // path layer il: LayerStart/StopHeight
  long long first[kMaxLayers + 1];             // first sample of path layer il; first[nl] = n_air
  long long n_ice;
};

// Device copy of the sampler constants (written by single_ray_kernel, read by path_kernel).
struct PathConsts {
  double summary[AIRICE_SINGLE_RAY_FIELDS];
  double L;
  double fstart[kMaxLayers];  // fDnfR(-LayerStartHeight, ...) of path layer il
  double off[kMaxLayers];     // LastRefracted_x entering path layer il
  double off_ice;             // LastRefracted_x after the air layers
  double fice0;               // fDnfR(0, A_ice, B_ice, C_ice, L)
};

// fDnfR (RayTracingFunctions.cc:293-302), pow(y,2) == y*y.
__device__ __forceinline__ double fDnfR(double x, double A, double B, double C, double L) {
  const double y = A + B * exp(C * x);
  return (L / C) * (1.0 / sqrt(A * A - L * L)) *
         (C * x - log(A * (A + B * exp(C * x)) - L * L + sqrt(A * A - L * L) * sqrt(y * y - L * L)));
}

__device__ __forceinline__ double B_air(const DevMedium& M, double z) {
  return sel5(M.B, air_layer(M, fabs(z)));
}
__device__ __forceinline__ double C_air(const DevMedium& M, double z) {  // +C (GetC_air)
  return -sel5(M.negC, air_layer(M, fabs(z)));
}
__device__ __forceinline__ double nz_air(const DevMedium& M, double z) {
  const double zabs = fabs(z);
  return M.A_air + B_air(M, zabs) * exp(-C_air(M, zabs) * zabs);
}
__device__ __forceinline__ double nz_ice(const DevMedium& M, double z) {
  z = fabs(z);
  return M.A_ice + M.B_ice * exp(M.negC_ice * z);
}

// GetRayOpticalPath (RayTracingFunctions.cc:349-369): the horizontal distance of a segment.
__device__ __forceinline__ double ray_path(const DevMedium& M, double A, double Rx, double Tx,
                                           double L, bool air) {
  double x1;
  if (air) {
    x1 = +fDnfR(Rx, A, B_air(M, Rx), -C_air(M, Rx), L) - fDnfR(Tx, A, B_air(M, Tx), -C_air(M, Tx), L);
    x1 *= -1;
  } else {
    x1 = +fDnfR(Rx, A, M.B_ice, M.negC_ice, L) - fDnfR(Tx, A, M.B_ice, M.negC_ice, L);
  }
  return x1;
}

// ftimeD, ice variant (RayTracingFunctions.cc:339-341)
__device__ __forceinline__ double ftimeD_ice(const DevMedium& M, double x, double A, double C,
                                             double L) {
  const double n = nz_ice(M, x);
  const double n2 = n * n;
  return (1.0 / (kSpeedC * C * sqrt(n2 - L * L))) *
         (n2 - L * L +
          (C * x - log(A * n - L * L + sqrt(A * A - L * L) * sqrt(n2 - L * L))) *
              (A * A * sqrt(n2 - L * L)) / sqrt(A * A - L * L) +
          A * sqrt(n2 - L * L) * log(n + sqrt(n2 - L * L)));
}

__global__ void single_ray_kernel(DevMedium M, PathPlan P, PathConsts* __restrict__ out) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const double r2d = M.r2d;
  double thd_air = 0.0, start_angle = 0.0, L = 0.0;
  // the air layer loop (.C:100-154)
  for (int il = P.top; il > P.bot - 1; --il) {
    const double start_h = (il == P.top) ? P.txh : M.atm[il + 1] - 0.00001;
    const double start_n = nz_air(M, start_h);
    const double stop_h = (il == P.bot) ? P.ice : M.atm[il];
    if (il == P.top) {
      // GetLayerHitPointPar (RayTracingFunctions.cc:399-514), air
      const double inc = (180 - P.launch) * M.d2r;
      const double nzRx = nz_air(M, stop_h), nzTx = nz_air(M, start_h);
      const double lang = asin((start_n / nzTx) * sin(inc));
      const double recv = asin((nz_air(M, start_h) * sin(lang)) / nz_air(M, stop_h));
      L = nzRx * sin(recv);
      thd_air += ray_path(M, M.A_air, stop_h, start_h, L, true);
      start_angle = recv * r2d;
    } else {
      const double rec = asin(L / nz_air(M, stop_h)) * r2d;
      thd_air += ray_path(M, M.A_air, stop_h, start_h, L, true);
      start_angle = rec;
    }
  }
  // GetIcePropagationPar (RayTracingFunctions.cc:661-679)
  const double thd_ice = ray_path(M, M.A_ice, P.depth, 0.0, L, false);
  const double recv_ice = asin(L / nz_ice(M, P.depth)) * r2d;
  const double t_ice = +ftimeD_ice(M, P.depth, M.A_ice, M.negC_ice, L) -
                       ftimeD_ice(M, 0.0, M.A_ice, M.negC_ice, L);
  out->summary[0] = thd_air;
  out->summary[1] = L;
  out->summary[2] = start_angle;
  out->summary[3] = thd_ice;
  out->summary[4] = recv_ice;
  out->summary[5] = t_ice;
  out->L = L;
  // sampler constants (.C:226-299): layerLs[il] == L for every layer, LvalueIce == L
  double last_x = 0.0;
  for (int il = 0; il < P.nl; ++il) {
    const double s = P.start[il];
    const double fs = fDnfR(-(s), M.A_air, B_air(M, -(s)), C_air(M, -(s)), L);
    out->fstart[il] = fs;
    out->off[il] = last_x;
    if (P.first[il + 1] > P.first[il]) {  // the layer's last sample sits at its stop height
      const double i = P.stop[il];
      last_x = fDnfR(-i, M.A_air, B_air(M, -i), C_air(M, -i), L) - fs + last_x;
    }
  }
  out->off_ice = last_x;
  out->fice0 = fDnfR(0, M.A_ice, M.B_ice, -M.negC_ice, L);
}

__global__ __launch_bounds__(kPathBlock) void path_kernel(DevMedium M, PathPlan P,
                                                           const PathConsts* __restrict__ c,
                                                           double* __restrict__ xs,
                                                           double* __restrict__ zs) {
  const long long k = (long long)blockIdx.x * kPathBlock + threadIdx.x;
  const long long n_air = P.first[P.nl];
  if (k >= n_air + P.n_ice) return;
  const double L = c->L;
  if (k < n_air) {
    int il = 0;
#pragma unroll
    for (int l = 1; l < kMaxLayers; ++l)
      if (l < P.nl && k >= P.first[l]) il = l;
    // i = LayerStartHeight - j equals the reference's repeated i = i - 1 (each step is exact)
    double i = P.start[il] - (double)(k - P.first[il]);
    if (i < P.stop[il]) i = P.stop[il];
    xs[k] = fDnfR(-i, M.A_air, B_air(M, -i), C_air(M, -i), L) - c->fstart[il] + c->off[il];
    zs[k] = i;
  } else {
    const int i = -(int)(k - n_air);
    xs[k] = c->off_ice - fDnfR((double)i, M.A_ice, M.B_ice, -M.negC_ice, L) + c->fice0;
    zs[k] = (double)i + P.ice;
  }
}

// Layer-skip scans (.C:60-86; RayTracingFunctions.cc:534-558)
int skip_above(const airice_medium* m, double txh) {
  int skip = 0;
  for (int il = m->max_layers; il > -1; il--) {
    // ATMLAY[il-1] is read only when the first test holds (txh < ATMLAY[0]/100 = 0 at il = 0)
    if (txh < m->atmlay_cm[il] / 100 && (il - 1 >= 0 ? txh >= m->atmlay_cm[il - 1] / 100 : false))
      il = -100;
    if (il > -1) skip++;
  }
  return skip;
}

int skip_below(const airice_medium* m, double ice) {
  int skip = 0;
  for (int il = 0; il < m->max_layers; il++) {
    if (ice >= m->atmlay_cm[il] / 100 && ice < m->atmlay_cm[il + 1] / 100) il = 100;
    if (il < m->max_layers) skip++;
  }
  return skip;
}

constexpr long long kMaxSamples = 1LL << 31;

int make_plan(const airice_medium* m, double depth, double launch, double txh, double ice,
              PathPlan* P, airice_single_ray_info* info) {
  std::memset(P, 0, sizeof(*P));
  P->txh = txh;
  P->ice = ice;
  P->depth = depth;
  P->launch = launch;
  const int sa = skip_above(m, txh), sb = skip_below(m, ice);
  P->top = m->max_layers - sa - 1;
  P->bot = sb;
  P->nl = m->max_layers - sa - sb;
  if (P->nl < 0) P->nl = 0;
  if (P->nl > kMaxLayers || P->top >= kMaxLayers) {
    set_error("single ray: %d path layers", P->nl);
    return AIRICE_EINVAL;
  }
  // sample ranges of the path loops (.C:226-299)
  long long n = 0;
  double last_height = 0;
  for (int il = 0; il < P->nl; ++il) {
    const double start = (il == 0) ? txh : last_height - 0.00001;
    const double stop = (il == P->nl - 1) ? ice : m->atmlay_cm[P->nl - il - 1] / 100;
    P->start[il] = start;
    P->stop[il] = stop;
    P->first[il] = n;
    // samples i = start, start-1, ... while i > stop-1, the last one clamped up to stop
    // (start - k is exact: every iterate is a multiple of ulp(start) no larger than start, so
    // the count is the number of k >= 0 with start - k > stop - 1, found with the loop's test)
    long long cnt = 0;
    if (start > stop - 1) {
      const double guess = std::floor(start - (stop - 1));
      if (!(guess < (double)kMaxSamples)) {
        set_error("single ray: path layer of %g samples", guess);
        return AIRICE_EINVAL;
      }
      cnt = (long long)guess;
      while (cnt > 0 && !(start - (double)(cnt - 1) > stop - 1)) --cnt;
      while (start - (double)cnt > stop - 1) ++cnt;
      last_height = (start - (double)(cnt - 1) < stop) ? stop : start - (double)(cnt - 1);
    }
    n += cnt;
  }
  for (int il = P->nl; il <= kMaxLayers; ++il) P->first[il] = n;
  // ice samples: for (int i = 0; i > -(depth+1); i--)
  const double lim = depth + 1;
  P->n_ice = (lim > 0) ? (long long)std::ceil(lim) : 0;
  if (!(P->n_ice < kMaxSamples) || !(n + P->n_ice < kMaxSamples)) {
    set_error("single ray: too many path samples");
    return AIRICE_EINVAL;
  }
  if (info != nullptr) {
    info->skip_above = sa;
    info->skip_below = sb;
    info->n_layers = P->nl;
    info->pad_ = 0;
    info->n_air = n;
    info->n_ice = P->n_ice;
  }
  return AIRICE_OK;
}

}  // namespace

int plan_single_ray(const airice_medium* m, double depth, double launch, double txh, double ice,
                    airice_single_ray_info* info) {
  PathPlan P;
  return make_plan(m, depth, launch, txh, ice, &P, info);
}

static_assert(sizeof(PathConsts) <= sizeof(double) * AIRICE_SINGLE_RAY_WORK,
              "AIRICE_SINGLE_RAY_WORK too small");

int launch_single_ray(const DevMedium& M, const airice_medium* m, double depth, double launch,
                      double txh, double ice, double* d_work, double* d_x, double* d_z,
                      size_t cap, hipStream_t st) {
  PathPlan P;
  int rc = make_plan(m, depth, launch, txh, ice, &P, nullptr);
  if (rc) return rc;
  const long long n = P.first[P.nl] + P.n_ice;
  if ((d_x != nullptr || d_z != nullptr) && (size_t)n > cap) {
    set_error("single ray: %lld path samples exceed capacity %zu", n, cap);
    return AIRICE_EINVAL;
  }
  PathConsts* c = reinterpret_cast<PathConsts*>(d_work);  // summary[] first
  count_launch(LC_SINGLE_RAY);
  hipLaunchKernelGGL(single_ray_kernel, dim3(1), dim3(64), 0, st, M, P, c);
  if (d_x != nullptr && d_z != nullptr && n > 0) {
    const unsigned grid = (unsigned)((n + kPathBlock - 1) / kPathBlock);
    count_launch(LC_PATH);
    hipLaunchKernelGGL(path_kernel, dim3(grid), dim3(kPathBlock), 0, st, M, P, c, d_x, d_z);
  }
  return hipGetLastError() == hipSuccess ? AIRICE_OK : AIRICE_EHIP;
}

}  // namespace airice
