// compat_multiray.cpp -- MultiRayAirIceRefraction:: C++ surface over the C-ABI
// (include/MultiRayAirIceRefraction.h).  Keeps the reference's globals and call semantics;
// every ray / solve is computed by the gfx950 kernels.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "MultiRayAirIceRefraction.h"
#include "airice.h"

// ---- reference globals (.cc:3-21) --------------------------------------------------------
double MaxAirTxHeight = 0;
double MinAirTxHeight = 0;
std::vector<std::vector<std::vector<float>>> AllTableAllAntData;
double AngleStepSize = 0.1;
double LoopStartAngle = 90.1;
double LoopStopAngle = 180.0;
int TotalAngleSteps = (int)std::floor((LoopStopAngle - LoopStartAngle) / AngleStepSize) + 1;
double HeightStepSize = 10;
double LoopStartHeight = 0;
double LoopStopHeight = 0;
int TotalHeightSteps = 0;

namespace {

std::mutex g_mu;
airice_medium g_medium;
bool g_have_medium = false;
double* g_scratch = nullptr;  // device scratch for scalar calls
constexpr size_t kScratch = 64;

void die(const char* what) {
  std::fprintf(stderr, "MultiRayAirIceRefraction: %s failed: %s\n", what, airice_last_error());
  std::abort();  // the reference has no error channel here; fail loudly, never fall back
}

const airice_medium& medium() {
  if (!g_have_medium) MultiRayAirIceRefraction::MakeAtmosphere();
  return g_medium;
}

double* scratch() {
  if (g_scratch == nullptr && hipMalloc(&g_scratch, kScratch * sizeof(double)) != hipSuccess)
    die("hipMalloc");
  return g_scratch;
}

}  // namespace

namespace MultiRayAirIceRefraction {

int MakeAtmosphere() {
  std::lock_guard<std::mutex> lock(g_mu);
  int rc = airice_atmosphere_load("Atmosphere.dat", AIRICE_VARIANT_MULTIRAY, &g_medium);
  if (rc != AIRICE_OK) {
    const char* env = std::getenv("AIRICE_ATMOSPHERE");
    if (env == nullptr || airice_atmosphere_load(env, AIRICE_VARIANT_MULTIRAY, &g_medium) != AIRICE_OK)
      die("MakeAtmosphere (Atmosphere.dat not found in the working directory or $AIRICE_ATMOSPHERE)");
  }
  g_have_medium = true;
  return 0;
}

double GetB_ice(double) { return medium().B_ice; }
double GetC_ice(double) { return medium().C_ice; }
double Getnz_ice(double z) { return airice_nz_ice(&medium(), z); }

static int layer_of(double z) {
  const airice_medium& m = medium();
  const double zabs = std::fabs(z);
  int which = 0;
  for (int l = 0; l < m.max_layers - 1; ++l)
    if (zabs < m.atmlay_cm[l + 1] / 100 && zabs >= m.atmlay_cm[l] / 100) {
      which = l;
      break;
    }
  if (zabs >= m.atmlay_cm[m.max_layers - 1] / 100) which = m.max_layers - 1;
  return which;
}
double GetB_air(double z) { return medium().B_air[layer_of(z)]; }
double GetC_air(double z) { return medium().C_air[layer_of(z)]; }
double Getnz_air(double z) { return airice_nz_air(&medium(), z); }

// Fresnel amplitude coefficients (.cc:267-337)
static void fresnel(double thetai, double ice, double& rS, double& tS, double& rP, double& tP) {
  const double n1 = Getnz_air(ice), n2 = Getnz_ice(0);
  const double a = (n1 / n2) * std::sin(thetai);
  const double sq = std::sqrt(1 - a * a);
  double num = n1 * std::cos(thetai) - n2 * sq, den = n1 * std::cos(thetai) + n2 * sq;
  rS = num / den;
  tS = 1 + num / den;
  num = n1 * sq - n2 * std::cos(thetai);
  den = n1 * sq + n2 * std::cos(thetai);
  rP = -(num) / (den);
  tP = (1 - (num / den)) * (n1 / n2);
  if (std::isnan(rS)) rS = 1;
  if (std::isnan(tS)) tS = 0;
  if (std::isnan(rP)) rP = 1;
  if (std::isnan(tP)) tP = 0;
}
double Refl_S(double t, double ice) { double a, b, c, d; fresnel(t, ice, a, b, c, d); return a; }
double Trans_S(double t, double ice) { double a, b, c, d; fresnel(t, ice, a, b, c, d); return b; }
double Refl_P(double t, double ice) { double a, b, c, d; fresnel(t, ice, a, b, c, d); return c; }
double Trans_P(double t, double ice) { double a, b, c, d; fresnel(t, ice, a, b, c, d); return d; }

double oneDLinearInterpolation(double x, double xa, double ya, double xb, double yb) {
  return ya + (yb - ya) * ((x - xa) / (xb - xa));  // .cc:992-995
}

void Air2IceRayTracing(double AirTxHeight, double HorizontalDistance, double IceLayerHeight,
                       double AntennaDepth, double StraightAngle, double dummy[20]) {
  const airice_medium& m = medium();
  std::lock_guard<std::mutex> lock(g_mu);
  double* d = scratch();
  double in[4] = {AirTxHeight, HorizontalDistance, AntennaDepth, StraightAngle};
  if (hipMemcpy(d, in, sizeof(in), hipMemcpyHostToDevice) != hipSuccess) die("hipMemcpy");
  if (airice_solve_launch(&m, AIRICE_VARIANT_MULTIRAY, IceLayerHeight, d, d + 1, d + 2, d + 3, 1,
                          d + 4, 1, nullptr, nullptr) != AIRICE_OK)
    die("Air2IceRayTracing");
  if (hipMemcpy(dummy, d + 4, sizeof(double) * AIRICE_SOLVE_FIELDS, hipMemcpyDeviceToHost) != hipSuccess)
    die("hipMemcpy");
}

void GetRayTracingSolutions(double RayLaunchAngleInAir, double AirTxHeight, double IceLayerHeight,
                            double AntennaDepth, double dummy[20], bool& InIce) {
  const airice_medium& m = medium();
  std::lock_guard<std::mutex> lock(g_mu);
  double* d = scratch();
  double in[2] = {RayLaunchAngleInAir, AirTxHeight};
  if (hipMemcpy(d, in, sizeof(in), hipMemcpyHostToDevice) != hipSuccess) die("hipMemcpy");
  if (airice_rays_launch(&m, d, d + 1, IceLayerHeight, AntennaDepth, InIce ? 1 : 0, 1, d + 2, 1,
                         nullptr) != AIRICE_OK)
    die("GetRayTracingSolutions");
  if (hipMemcpy(dummy, d + 2, sizeof(double) * AIRICE_RAY_FIELDS, hipMemcpyDeviceToHost) != hipSuccess)
    die("hipMemcpy");
}

bool GetHorizontalDistanceToIntersectionPoint(
    double SrcHeightASL, double HorizontalDistanceToRx, double RxDepthBelowIceBoundary,
    double IceLayerHeight, double& opticalPathLengthInIce, double& opticalPathLengthInAir,
    double& geometricalPathLengthInIce, double& geometricalPathLengthInAir, double& launchAngle,
    double& horizontalDistanceToIntersectionPoint, double& transmissionCoefficientS,
    double& transmissionCoefficientP, double& RecievedAngleInIce) {
  const airice_medium& m = medium();
  std::lock_guard<std::mutex> lock(g_mu);
  double* d = scratch();
  double in[3] = {SrcHeightASL, HorizontalDistanceToRx, RxDepthBelowIceBoundary};
  if (hipMemcpy(d, in, sizeof(in), hipMemcpyHostToDevice) != hipSuccess) die("hipMemcpy");
  uint8_t* ok = reinterpret_cast<uint8_t*>(d + 12);
  if (airice_hdtip_launch(&m, d, d + 1, d + 2, IceLayerHeight, 1, d + 3, 1, ok, nullptr) != AIRICE_OK)
    die("GetHorizontalDistanceToIntersectionPoint");
  double o[10];
  if (hipMemcpy(o, d + 3, sizeof(double) * 10, hipMemcpyDeviceToHost) != hipSuccess) die("hipMemcpy");
  opticalPathLengthInIce = o[0];
  opticalPathLengthInAir = o[1];
  geometricalPathLengthInIce = o[2];
  geometricalPathLengthInAir = o[3];
  launchAngle = o[4];
  horizontalDistanceToIntersectionPoint = o[5];
  transmissionCoefficientS = o[6];
  transmissionCoefficientP = o[7];
  RecievedAngleInIce = o[8];
  const uint8_t flag = reinterpret_cast<const uint8_t*>(&o[9])[0];
  return flag != 0;
}

int MakeRayTracingTable(double AntennaDepth, double IceLayerHeight, int AntennaNumber) {
  (void)AntennaNumber;  // the reference appends in call order (.cc:2136)
  MakeAtmosphere();     // the reference re-reads the atmosphere on every table (.cc:2039)
  const airice_medium& m = medium();
  airice_grid g;
  if (airice_grid_init(&g, AntennaDepth, IceLayerHeight, HeightStepSize, LoopStartAngle,
                       LoopStopAngle, AngleStepSize) != AIRICE_OK)
    die("MakeRayTracingTable grid");
  g.angle_steps = TotalAngleSteps;  // the global, computed at static init (.cc:15)
  LoopStartHeight = g.start_height;
  LoopStopHeight = g.stop_height;
  TotalHeightSteps = g.height_steps;
  const size_t n = (size_t)g.height_steps * (size_t)g.angle_steps;
  float* dt = nullptr;
  if (hipMalloc(&dt, sizeof(float) * 11 * n) != hipSuccess) die("hipMalloc table");
  if (airice_table_launch(&m, &g, 0, g.height_steps, dt, nullptr, n, nullptr) != AIRICE_OK)
    die("MakeRayTracingTable");
  std::vector<std::vector<float>> cols(11, std::vector<float>(n));
  for (int c = 0; c < 11; ++c)
    if (hipMemcpy(cols[c].data(), dt + (size_t)c * n, sizeof(float) * n, hipMemcpyDeviceToHost) !=
        hipSuccess)
      die("hipMemcpy table");
  (void)hipFree(dt);
  AllTableAllAntData.push_back(std::move(cols));
  return 0;
}

}  // namespace MultiRayAirIceRefraction
