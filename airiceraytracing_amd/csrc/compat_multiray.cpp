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

// HBM copy of AllTableAllAntData[i]: adopted from MakeRayTracingTable, or uploaded when the
// host table at that index is not the one last seen (a caller-filled or replaced table).
struct DevTable {
  const float* host0 = nullptr;  // AllTableAllAntData[i][0].data() when mirrored
  size_t n = 0;
  float* dev = nullptr;
  float* packed = nullptr;  // airice_lookup_pack copy, made at the first lookup
};
std::vector<DevTable> g_tables;

const float* device_table(int index, size_t* n_out) {
  if (index < 0 || index >= (int)AllTableAllAntData.size()) {
    std::fprintf(stderr, "MultiRayAirIceRefraction: no table %d (%zu made)\n", index,
                 AllTableAllAntData.size());
    std::abort();  // the reference indexes out of range here (UB); fail loudly instead
  }
  const std::vector<std::vector<float>>& cols = AllTableAllAntData[index];
  if (cols.size() < AIRICE_TABLE_COLUMNS || cols[0].empty()) die("table lookup (malformed table)");
  const size_t n = cols[0].size();
  if (g_tables.size() <= (size_t)index) g_tables.resize(index + 1);
  DevTable& t = g_tables[index];
  *n_out = n;
  if (t.dev != nullptr && t.host0 == cols[0].data() && t.n == n) return t.dev;
  if (t.dev != nullptr) (void)hipFree(t.dev);
  if (t.packed != nullptr) (void)hipFree(t.packed);
  t.dev = nullptr;
  t.packed = nullptr;
  if (hipMalloc(&t.dev, sizeof(float) * AIRICE_TABLE_COLUMNS * n) != hipSuccess) die("hipMalloc");
  for (int c = 0; c < AIRICE_TABLE_COLUMNS; ++c) {
    if (cols[c].size() != n) die("table lookup (ragged table)");
    if (hipMemcpy(t.dev + (size_t)c * n, cols[c].data(), sizeof(float) * n,
                  hipMemcpyHostToDevice) != hipSuccess)
      die("hipMemcpy table");
  }
  t.host0 = cols[0].data();
  t.n = n;
  return t.dev;
}

airice_lookup_table lookup_desc(const float* dev, size_t n) {
  airice_lookup_table t;
  t.entries = nullptr;
  t.table = dev;
  t.ld = n;
  t.n_entries = n;
  t.loop_stop_height = LoopStopHeight;  // globals of the last table made (.cc:1035-1039)
  t.height_step = HeightStepSize;
  t.total_height_steps = TotalHeightSteps;
  t.total_angle_steps = TotalAngleSteps;
  return t;
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
  AllTableAllAntData.push_back(std::move(cols));
  // keep the HBM copy for the lookups (moving the column vectors keeps their storage)
  const size_t index = AllTableAllAntData.size() - 1;
  if (g_tables.size() <= index) g_tables.resize(index + 1);
  if (g_tables[index].dev != nullptr) (void)hipFree(g_tables[index].dev);
  if (g_tables[index].packed != nullptr) (void)hipFree(g_tables[index].packed);
  g_tables[index].packed = nullptr;
  g_tables[index].dev = dt;
  g_tables[index].host0 = AllTableAllAntData[index][0].data();
  g_tables[index].n = n;
  return 0;
}

bool TableLookup(double SrcHeightASL, double HorizontalDistanceToRx,
                 double RxDepthBelowIceBoundary, double IceLayerHeight, int TableIndex,
                 double& opticalPathLengthInIce, double& opticalPathLengthInAir,
                 double& geometricalPathLengthInIce, double& geometricalPathLengthInAir,
                 double& launchAngle, double& horizontalDistanceToIntersectionPoint,
                 double& transmissionCoefficientS, double& transmissionCoefficientP,
                 double& RecievedAngleInIce) {
  const double src[1] = {SrcHeightASL}, dist[1] = {HorizontalDistanceToRx},
               dep[1] = {RxDepthBelowIceBoundary};
  double o[9];
  bool ok = false;
  TableLookupBatch(src, dist, dep, IceLayerHeight, TableIndex, 1, o, &ok);
  opticalPathLengthInIce = o[0];
  opticalPathLengthInAir = o[1];
  geometricalPathLengthInIce = o[2];
  geometricalPathLengthInAir = o[3];
  launchAngle = o[4];
  horizontalDistanceToIntersectionPoint = o[5];
  transmissionCoefficientS = o[6];
  transmissionCoefficientP = o[7];
  RecievedAngleInIce = o[8];
  return ok;
}

void TableLookupBatch(const double* SrcHeightASL, const double* HorizontalDistanceToRx,
                      const double* RxDepthBelowIceBoundary, double IceLayerHeight, int TableIndex,
                      size_t n, double* out9, bool* ok) {
  const airice_medium& m = medium();
  std::lock_guard<std::mutex> lock(g_mu);
  size_t entries = 0;
  const float* dev = device_table(TableIndex, &entries);
  // MaxAirTxHeight / MinAirTxHeight globals (.cc:1359-1360)
  MaxAirTxHeight = AllTableAllAntData[TableIndex][0][0];
  MinAirTxHeight = AllTableAllAntData[TableIndex][0][entries - 1];
  if (n == 0) return;
  // one device block: src | dist | depth | out (9 columns) | ok | flags
  const size_t bytes = sizeof(double) * 12 * n + 2 * n;
  const bool small = bytes <= kScratch * sizeof(double);
  double* d = small ? scratch() : nullptr;
  if (!small && hipMalloc(&d, bytes) != hipSuccess) die("hipMalloc");
  if (hipMemcpy(d, SrcHeightASL, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d + n, HorizontalDistanceToRx, sizeof(double) * n, hipMemcpyHostToDevice) !=
          hipSuccess ||
      hipMemcpy(d + 2 * n, RxDepthBelowIceBoundary, sizeof(double) * n, hipMemcpyHostToDevice) !=
          hipSuccess)
    die("hipMemcpy");
  uint8_t* dok = reinterpret_cast<uint8_t*>(d + 12 * n);
  uint8_t* dfl = dok + n;
  airice_lookup_table t = lookup_desc(dev, entries);
  DevTable& dt = g_tables[TableIndex];
  if (dt.packed == nullptr) {
    if (hipMalloc(&dt.packed, sizeof(float) * AIRICE_LOOKUP_ENTRY_FLOATS * entries) != hipSuccess ||
        airice_lookup_pack(&t, dt.packed, nullptr) != AIRICE_OK)
      die("airice_lookup_pack");
  }
  t.entries = dt.packed;
  if (airice_table_lookup_launch(&m, &t, d, d + n, d + 2 * n, IceLayerHeight, n, d + 3 * n, n,
                                 dok, dfl, nullptr) != AIRICE_OK)
    die("GetHorizontalDistanceToIntersectionPoint_Table");
  std::vector<double> soa(9 * n);
  std::vector<uint8_t> hok(n);
  if (hipMemcpy(soa.data(), d + 3 * n, sizeof(double) * 9 * n, hipMemcpyDeviceToHost) !=
          hipSuccess ||
      hipMemcpy(hok.data(), dok, n, hipMemcpyDeviceToHost) != hipSuccess)
    die("hipMemcpy");
  if (!small) (void)hipFree(d);
  for (size_t i = 0; i < n; ++i) {
    for (int c = 0; c < 9; ++c) out9[i * 9 + c] = soa[(size_t)c * n + i];
    ok[i] = hok[i] != 0;
  }
}

}  // namespace MultiRayAirIceRefraction
