// compat_multiray.cpp -- MultiRayAirIceRefraction:: C++ surface over the C-ABI
// (include/MultiRayAirIceRefraction.h).  Keeps the reference's globals and call semantics.
// Ray quantities and solves run on the GPU: batches through the batch kernels, one-query calls
// through the current device's pinned scalar slot (ScalarCall, airice_runtime.cpp: the kernels
// read their inputs from and write their outputs to pinned host memory, one synchronisation per
// call).  Table walks (_Table, GetParValues, FindClosest*) run the batch lookup kernel's own
// code (airice_lookup.hpp) on the host against the caller's host columns.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <initializer_list>
#include <mutex>
#include <vector>

#include "MultiRayAirIceRefraction.h"
#include "airice.h"
#include "airice_internal.h"
#include "airice_lookup.hpp"
#include "compat_common.h"

// The caller owns these (reference .h:23-24, RunMultiRayCode.C:3-4); only _Table reads them.
// Weak references: a process that never defines them (a ctypes user of the C-ABI) still loads
// the library, and _Table then skips the antenna remap.
#pragma weak AntennaDepths
#pragma weak AntennaTableAlreadyMade

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

// ---- namespace data (.h:33-84): one shared copy -------------------------------------------
namespace MultiRayAirIceRefraction {
std::vector<std::vector<double>> nh_data;
std::vector<std::vector<double>> lognh_data;
std::vector<std::vector<double>> h_data;
std::vector<double> GridPositionH;
std::vector<double> GridPositionTh;
std::vector<double> GridZValue[10];
double GridStartTh = 90.05;
double GridStopTh = 179.95;
double GridStepSizeH_O = 25;
double GridStepSizeTh_O = 0.01;
double GridWidthH = 1000;
double GridWidthTh = GridStopTh - GridStartTh;
int GridPoints = 100;
int TotalStepsH_O = 100;
int TotalStepsTh_O = 100;
double GridStartH = 1000;
double GridStopH = 100000;
double ATMLAY[5];
double abc[5][3];
double C_air[5];
double B_air[5];
double A_ice = A_ice_def;
double B_ice = B_ice_def;
double C_ice = C_ice_def;
int MaxLayers = 0;
}  // namespace MultiRayAirIceRefraction

namespace {

namespace MR = MultiRayAirIceRefraction;

std::mutex g_mu;  // the medium and the HBM table copies
airice_medium g_medium;     // the parse of Atmosphere.dat (N0, profile size)
bool g_have_medium = false;
bool g_ns_filled = false;   // MakeAtmosphere has filled the namespace data

[[noreturn]] void die(const char* what) {
  std::fprintf(stderr, "MultiRayAirIceRefraction: %s failed: %s\n", what, airice_last_error());
  std::abort();  // the reference has no error channel here; fail loudly, never fall back
}

std::string atmosphere_text() { return airice_compat::atmosphere_text("MultiRayAirIceRefraction"); }

// The medium of the next call: the parse of the file with the namespace's current air model
// (ATMLAY, B_air, C_air, MaxLayers once MakeAtmosphere has filled them) and ice model (A_ice /
// B_ice / C_ice) -- mutable namespace variables the reference reads at every call.  Before any
// MakeAtmosphere the file is parsed on first use.
airice_medium medium() {
  std::lock_guard<std::mutex> lock(g_mu);
  if (!g_have_medium) {
    const std::string text = atmosphere_text();
    if (airice_atmosphere_parse(text.data(), text.size(), AIRICE_VARIANT_MULTIRAY, &g_medium) !=
        AIRICE_OK)
      die("MakeAtmosphere");
    g_have_medium = true;
  }
  airice_medium m = g_medium;
  if (g_ns_filled) airice_compat::apply_namespace(m, MR::ATMLAY, MR::B_air, MR::C_air, MR::MaxLayers);
  m.A_ice = MR::A_ice;
  m.B_ice = MR::B_ice;
  m.C_ice = MR::C_ice;
  return m;
}

// one GPU evaluation of a ray-layer quantity (AIRICE_RTF_* / AIRICE_MR_* op)
void ray_op(int op, std::initializer_list<double> args, double* out, size_t n_out) {
  const airice_medium m = medium();
  const std::vector<double> a(args);
  if (airice_rtf_eval(&m, op, a.data(), a.size(), out, n_out) != AIRICE_OK) die("ray layer");
}

double ray_op1(int op, std::initializer_list<double> args) {
  double r = 0;
  ray_op(op, args, &r, 1);
  return r;
}

// ---- tables --------------------------------------------------------------------------------
const std::vector<std::vector<float>>& host_table(int index) {
  if (index < 0 || index >= (int)AllTableAllAntData.size()) {
    std::fprintf(stderr, "MultiRayAirIceRefraction: no table %d (%zu made)\n", index,
                 AllTableAllAntData.size());
    std::abort();  // the reference indexes out of range here (UB); fail loudly instead
  }
  const std::vector<std::vector<float>>& cols = AllTableAllAntData[index];
  if (cols.size() < AIRICE_TABLE_COLUMNS || cols[0].empty()) die("table lookup (malformed table)");
  for (int c = 1; c < AIRICE_TABLE_COLUMNS; ++c)
    if (cols[c].size() != cols[0].size()) die("table lookup (ragged table)");
  return cols;
}

// The lookup's view of a host table and the grid globals of the last table made (.cc:1035-1039)
airice::LkTable host_lk(const std::vector<std::vector<float>>& cols) {
  airice::LkTable T;
  for (int c = 0; c < AIRICE_TABLE_COLUMNS; ++c) T.col[c] = cols[c].data();
  T.e = nullptr;
  T.rows = 0;
  T.n = (long long)cols[0].size();
  T.stop_h = LoopStopHeight;
  T.step_h = HeightStepSize;
  T.hsteps = TotalHeightSteps;
  T.asteps = TotalAngleSteps;
  return T;
}

// Cheap content fingerprint of a host table: the column buffers, their length and 64 sampled
// entries per column.  The HBM copy of a table is reused only while this is unchanged: a table the
// caller replaced, resized or refilled is uploaded again, but an in-place edit of entries other
// than the sampled ones is NOT detected (hashing every entry would cost more than the lookups).
uint64_t table_fingerprint(const std::vector<std::vector<float>>& cols) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&h](uint64_t v) {
    h ^= v;
    h *= 1099511628211ull;
  };
  const size_t n = cols[0].size();
  mix(n);
  for (int c = 0; c < AIRICE_TABLE_COLUMNS; ++c) {
    mix(reinterpret_cast<uintptr_t>(cols[c].data()));
    for (size_t k = 0; k < 64; ++k) {
      uint32_t bits;
      std::memcpy(&bits, &cols[c][(n - 1) * k / 63], 4);
      mix(bits);
    }
  }
  return h;
}

// HBM copy of AllTableAllAntData[i] for the batch lookup: the copy MakeRayTracingTable left
// behind, or an upload.  A table whose fingerprint changed since (a caller-filled, replaced or
// resized table) is uploaded again.
struct DevTable {
  uint64_t fp = 0;
  size_t n = 0;
  float* dev = nullptr;
  float* packed = nullptr;  // airice_lookup_pack copy, made at the first batch lookup
  int packed_asteps = 0;    // the TotalAngleSteps its row records were folded with
};
std::vector<DevTable> g_tables;

void drop(DevTable& t) {
  if (t.dev != nullptr) (void)hipFree(t.dev);
  if (t.packed != nullptr) (void)hipFree(t.packed);
  t = DevTable();
}

DevTable& device_table(int index) {
  const std::vector<std::vector<float>>& cols = host_table(index);
  const size_t n = cols[0].size();
  if (g_tables.size() <= (size_t)index) g_tables.resize(index + 1);
  DevTable& t = g_tables[index];
  const uint64_t fp = table_fingerprint(cols);
  if (t.dev != nullptr && t.fp == fp && t.n == n) return t;
  drop(t);
  if (hipMalloc(&t.dev, sizeof(float) * AIRICE_TABLE_COLUMNS * n) != hipSuccess) die("hipMalloc");
  for (int c = 0; c < AIRICE_TABLE_COLUMNS; ++c)
    if (hipMemcpy(t.dev + (size_t)c * n, cols[c].data(), sizeof(float) * n,
                  hipMemcpyHostToDevice) != hipSuccess)
      die("hipMemcpy table");
  t.fp = fp;
  t.n = n;
  return t;
}

void set_minmax(const std::vector<std::vector<float>>& cols) {  // .cc:1357-1360 / 1175-1177
  MaxAirTxHeight = cols[0][0];
  MinAirTxHeight = cols[0][cols[0].size() - 1];
}

}  // namespace

namespace MultiRayAirIceRefraction {

// ---- atmosphere (.cc:24-213, 920-942) ------------------------------------------------------
int readATMpar() {
  airice_compat::read_atm_par(atmosphere_text(), ATMLAY, abc);
  return 0;
}

int readnhFromFile() {
  MaxLayers = airice_compat::read_nh(atmosphere_text(), ATMLAY, h_data, nh_data, lognh_data);
  if (MaxLayers == 0) {
    std::fprintf(stderr, "MultiRayAirIceRefraction: no refractive-index profile in "
                         "Atmosphere.dat\n");
    std::abort();
  }
  return 0;
}

// N0 from the natural cubic spline of the profile at 0 m, then B_air chained for continuity
// (.cc:193-213): the library's parse of the same file does exactly this
// over the namespace's ATMLAY / abc
int FillInAirRefractiveIndex() {
  const std::string text = atmosphere_text();
  std::lock_guard<std::mutex> lock(g_mu);
  if (airice_atmosphere_parse(text.data(), text.size(), AIRICE_VARIANT_MULTIRAY, &g_medium) !=
      AIRICE_OK)
    die("FillInAirRefractiveIndex");
  g_have_medium = true;
  airice_compat::fill_air_index(ATMLAY, abc, A_air, g_medium.N0, C_air, B_air);
  return 0;
}

std::vector<double> flatten(const std::vector<std::vector<double>>& v) {
  return airice_compat::flatten(v);
}

int MakeAtmosphere() {
  readATMpar();
  readnhFromFile();
  FillInAirRefractiveIndex();
  std::lock_guard<std::mutex> lock(g_mu);
  g_ns_filled = true;
  return 0;
}

// GetB_ice / GetC_ice (.cc:150-185; TransitionBoundary is 0) and the air model scan (.cc:216-263)
double GetB_ice(double) { return B_ice; }
double GetC_ice(double) { return C_ice; }
double Getnz_ice(double z) {
  const airice_medium m = medium();
  return airice_nz_ice(&m, z);
}

static int layer_of(double z) {  // the GetB_air / GetC_air scan (.cc:216-257)
  const airice_medium m = medium();
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
double Getnz_air(double z) {
  const airice_medium m = medium();
  return airice_nz_air(&m, z);
}

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

// ---- the ray layer (.cc:377-917) on the GPU ------------------------------------------------
double fDnfR(double x, void* params) {
  const fDnfR_params* p = static_cast<const fDnfR_params*>(params);
  return ray_op1(AIRICE_RTF_FDNFR, {x, p->a, p->b, p->c, p->l});
}

double ftimeD(double x, void* params) {
  const ftimeD_params* p = static_cast<const ftimeD_params*>(params);
  return ray_op1(AIRICE_RTF_FTIMED, {x, p->a, p->b, p->c, p->speedc, p->l, (double)p->airorice});
}

double fpathD(double x, void* params) {
  const ftimeD_params* p = static_cast<const ftimeD_params*>(params);
  return ray_op1(AIRICE_MR_FPATHD, {x, p->a, p->b, p->c, p->speedc, p->l});
}

double GetRayHorizontalPath(double A, double RxDepth, double TxDepth, double Lvalue, int AirOrIce) {
  return ray_op1(AIRICE_RTF_OPTICAL_PATH, {A, RxDepth, TxDepth, Lvalue, (double)AirOrIce});
}

double GetRayPropagationTime(double A, double RxDepth, double TxDepth, double Lvalue,
                             int AirOrIce) {
  return ray_op1(AIRICE_RTF_PROPAGATION_TIME, {A, RxDepth, TxDepth, Lvalue, (double)AirOrIce});
}

double GetRayGeometricPath(double A, double RxDepth, double TxDepth, double Lvalue, int AirOrIce) {
  return ray_op1(AIRICE_MR_GEOMETRIC_PATH, {A, RxDepth, TxDepth, Lvalue, (double)AirOrIce});
}

double* GetLayerHitPointPar(double n_layer1, double RxDepth, double TxDepth, double IncidentAng,
                            int AirOrIce) {
  double* out = new double[5];
  ray_op(AIRICE_MR_HIT_POINT, {n_layer1, RxDepth, TxDepth, IncidentAng, (double)AirOrIce}, out,
         5);
  return out;
}

double* GetAirPropagationPar(double LaunchAngle, double AirTxHeight, double IceLayerHeight) {
  const int n = 5 * medium().max_layers + 2;
  double* out = new double[n];
  ray_op(AIRICE_MR_AIR_PROPAGATION, {LaunchAngle, AirTxHeight, IceLayerHeight}, out, n);
  return out;
}

double* GetIcePropagationPar(double IncidentAngleonIce, double IceLayerHeight, double AntennaDepth,
                             double Lvalue) {
  double* out = new double[5];
  ray_op(AIRICE_MR_ICE_PROPAGATION, {IncidentAngleonIce, IceLayerHeight, AntennaDepth, Lvalue},
         out, 5);
  return out;
}

double MinimizeforLaunchAngle(double x, void* params) {
  const MinforLAng_params* p = static_cast<const MinforLAng_params*>(params);
  return ray_op1(AIRICE_MR_MIN_LAUNCH,
                 {x, p->airtxheight, p->icelayerheight, p->antennadepth, p->horizontaldistance});
}

// ---- one-query solves: one launch chain through the scalar slot ----------------------------
void Air2IceRayTracing(double AirTxHeight, double HorizontalDistance, double IceLayerHeight,
                       double AntennaDepth, double StraightAngle, double dummy[20]) {
  const airice_medium m = medium();
  if (airice::scalar_on_host()) {  // one query: on the host (airice_scalar_mode)
    const double in[4] = {AirTxHeight, HorizontalDistance, AntennaDepth, StraightAngle};
    if (airice::solve_query_host(&m, AIRICE_VARIANT_MULTIRAY, IceLayerHeight, in, true, dummy,
                                 nullptr) != AIRICE_OK)
      die("Air2IceRayTracing");
    return;
  }
  airice::ScalarCall call;
  if (!call.ok()) die("Air2IceRayTracing");
  airice::ScalarSlot& s = call.slot();
  s.h[0] = AirTxHeight;
  s.h[1] = HorizontalDistance;
  s.h[2] = AntennaDepth;
  s.h[3] = StraightAngle;
  call.arm(s.h, 4);
  if (airice_solve_launch(&m, AIRICE_VARIANT_MULTIRAY, IceLayerHeight, s.d, s.d + 1, s.d + 2,
                          s.d + 3, 1, s.d + 4, 1, nullptr, s.st) != AIRICE_OK ||
      call.sync() != AIRICE_OK)
    die("Air2IceRayTracing");
  std::memcpy(dummy, s.h + 4, sizeof(double) * AIRICE_SOLVE_FIELDS);
}

void GetRayTracingSolutions(double RayLaunchAngleInAir, double AirTxHeight, double IceLayerHeight,
                            double AntennaDepth, double dummy[20], bool& InIce) {
  const airice_medium m = medium();
  if (airice_scalar_mode(-1) == AIRICE_SCALAR_HOST) {  // one ray: on the host (airice_rays_host)
    if (airice_rays_host(&m, &RayLaunchAngleInAir, &AirTxHeight, IceLayerHeight, AntennaDepth,
                         InIce ? 1 : 0, 1, dummy, 1) != AIRICE_OK)
      die("GetRayTracingSolutions");
    return;
  }
  airice::ScalarCall call;
  if (!call.ok()) die("GetRayTracingSolutions");
  airice::ScalarSlot& s = call.slot();
  s.h[0] = RayLaunchAngleInAir;
  s.h[1] = AirTxHeight;
  call.arm(s.h, 2);
  if (airice_rays_launch(&m, s.d, s.d + 1, IceLayerHeight, AntennaDepth, InIce ? 1 : 0, 1,
                         s.d + 2, 1, s.st) != AIRICE_OK ||
      call.sync() != AIRICE_OK)
    die("GetRayTracingSolutions");
  std::memcpy(dummy, s.h + 2, sizeof(double) * AIRICE_RAY_FIELDS);
}

bool GetHorizontalDistanceToIntersectionPoint(
    double SrcHeightASL, double HorizontalDistanceToRx, double RxDepthBelowIceBoundary,
    double IceLayerHeight, double& opticalPathLengthInIce, double& opticalPathLengthInAir,
    double& geometricalPathLengthInIce, double& geometricalPathLengthInAir, double& launchAngle,
    double& horizontalDistanceToIntersectionPoint, double& transmissionCoefficientS,
    double& transmissionCoefficientP, double& RecievedAngleInIce) {
  const airice_medium m = medium();
  if (airice::scalar_on_host()) {  // one query: on the host (airice_scalar_mode)
    const double in[3] = {SrcHeightASL, HorizontalDistanceToRx, RxDepthBelowIceBoundary};
    double o[9];
    uint8_t ok = 0;
    if (airice::hdtip_query_host(&m, IceLayerHeight, in, o, &ok) != AIRICE_OK)
      die("GetHorizontalDistanceToIntersectionPoint");
    opticalPathLengthInIce = o[0];
    opticalPathLengthInAir = o[1];
    geometricalPathLengthInIce = o[2];
    geometricalPathLengthInAir = o[3];
    launchAngle = o[4];
    horizontalDistanceToIntersectionPoint = o[5];
    transmissionCoefficientS = o[6];
    transmissionCoefficientP = o[7];
    RecievedAngleInIce = o[8];
    return ok != 0;
  }
  airice::ScalarCall call;
  if (!call.ok()) die("GetHorizontalDistanceToIntersectionPoint");
  airice::ScalarSlot& s = call.slot();
  s.h[0] = SrcHeightASL;
  s.h[1] = HorizontalDistanceToRx;
  s.h[2] = RxDepthBelowIceBoundary;
  uint8_t* ok_h = reinterpret_cast<uint8_t*>(s.h + 12);
  uint8_t* ok_d = reinterpret_cast<uint8_t*>(s.d + 12);
  call.arm(s.h, 3);
  if (airice_hdtip_launch(&m, s.d, s.d + 1, s.d + 2, IceLayerHeight, 1, s.d + 3, 1, ok_d, s.st) !=
          AIRICE_OK ||
      call.sync() != AIRICE_OK)
    die("GetHorizontalDistanceToIntersectionPoint");
  const double* o = s.h + 3;
  opticalPathLengthInIce = o[0];
  opticalPathLengthInAir = o[1];
  geometricalPathLengthInIce = o[2];
  geometricalPathLengthInAir = o[3];
  launchAngle = o[4];
  horizontalDistanceToIntersectionPoint = o[5];
  transmissionCoefficientS = o[6];
  transmissionCoefficientP = o[7];
  RecievedAngleInIce = o[8];
  return ok_h[0] != 0;
}

// ---- MakeRayTracingTable (.cc:2019-2158) ---------------------------------------------------
int MakeRayTracingTable(double AntennaDepth, double IceLayerHeight, int AntennaNumber) {
  (void)AntennaNumber;  // the reference appends in call order (.cc:2136)
  MakeAtmosphere();     // the reference re-reads the atmosphere on every table (.cc:2039)
  const airice_medium m = medium();
  airice_grid g;
  if (airice_grid_init(&g, AntennaDepth, IceLayerHeight, HeightStepSize, LoopStartAngle,
                       LoopStopAngle, AngleStepSize) != AIRICE_OK)
    die("MakeRayTracingTable grid");
  g.angle_steps = TotalAngleSteps;  // the global, computed at static init (.cc:15)
  LoopStartHeight = g.start_height;
  LoopStopHeight = g.stop_height;
  TotalHeightSteps = g.height_steps;
  // rows with Tx <= 0 are skipped (.cc:2082): the table holds g.table_rows rows
  const size_t n = (size_t)g.table_rows * (size_t)g.angle_steps;
  float* dt = nullptr;
  if (n > 0 && hipMalloc(&dt, sizeof(float) * 11 * n) != hipSuccess) die("hipMalloc table");
  if (n > 0 && airice_table_launch(&m, &g, 0, g.table_rows, dt, nullptr, n, nullptr) != AIRICE_OK)
    die("MakeRayTracingTable");
  std::vector<std::vector<float>> cols(11, std::vector<float>(n));
  for (int c = 0; c < 11 && n > 0; ++c)
    if (hipMemcpy(cols[c].data(), dt + (size_t)c * n, sizeof(float) * n, hipMemcpyDeviceToHost) !=
        hipSuccess)
      die("hipMemcpy table");
  AllTableAllAntData.push_back(std::move(cols));
  // keep the HBM copy for batch lookups (moving the column vectors keeps their storage)
  std::lock_guard<std::mutex> lock(g_mu);
  const size_t index = AllTableAllAntData.size() - 1;
  if (g_tables.size() <= index) g_tables.resize(index + 1);
  drop(g_tables[index]);
  if (n > 0) {
    g_tables[index].dev = dt;
    g_tables[index].n = n;
    g_tables[index].fp = table_fingerprint(AllTableAllAntData[index]);
  }
  return 0;
}

int MakeRayTracingTables(const std::vector<double>& AntennaDepth, double IceLayerHeight) {
  const size_t na = AntennaDepth.size();
  if (na == 0) return 0;
  MakeAtmosphere();
  const airice_medium m = medium();
  std::vector<airice_grid> grids(na);
  std::vector<float*> dev(na, nullptr);
  std::vector<size_t> n(na);
  for (size_t a = 0; a < na; ++a) {
    airice_grid& g = grids[a];
    if (airice_grid_init(&g, AntennaDepth[a], IceLayerHeight, HeightStepSize, LoopStartAngle,
                         LoopStopAngle, AngleStepSize) != AIRICE_OK)
      die("MakeRayTracingTables grid");
    g.angle_steps = TotalAngleSteps;  // the global, computed at static init (.cc:15)
    n[a] = (size_t)g.table_rows * (size_t)g.angle_steps;
    if (n[a] > 0 && hipMalloc(&dev[a], sizeof(float) * 11 * n[a]) != hipSuccess)
      die("hipMalloc table");
  }
  // antennas whose table is empty (every Tx row skipped) take no part in the launch
  std::vector<airice_grid> lg;
  std::vector<float*> lt;
  std::vector<size_t> ll;
  for (size_t a = 0; a < na; ++a)
    if (n[a] > 0) {
      lg.push_back(grids[a]);
      lt.push_back(dev[a]);
      ll.push_back(n[a]);
    }
  for (size_t s = 0; s < lg.size(); s += 32) {
    const int cnt = (int)std::min<size_t>(32, lg.size() - s);
    if (airice_table_launch_multi(&m, lg.data() + s, cnt, lt.data() + s, ll.data() + s, nullptr) !=
        AIRICE_OK)
      die("MakeRayTracingTables");
  }
  for (size_t a = 0; a < na; ++a) {
    std::vector<std::vector<float>> cols(11, std::vector<float>(n[a]));
    for (int c = 0; c < 11 && n[a] > 0; ++c)
      if (hipMemcpy(cols[c].data(), dev[a] + (size_t)c * n[a], sizeof(float) * n[a],
                    hipMemcpyDeviceToHost) != hipSuccess)
        die("hipMemcpy table");
    AllTableAllAntData.push_back(std::move(cols));
    std::lock_guard<std::mutex> lock(g_mu);
    const size_t index = AllTableAllAntData.size() - 1;
    if (g_tables.size() <= index) g_tables.resize(index + 1);
    drop(g_tables[index]);
    if (n[a] > 0) {
      g_tables[index].dev = dev[a];
      g_tables[index].n = n[a];
      g_tables[index].fp = table_fingerprint(AllTableAllAntData[index]);
    }
  }
  const airice_grid& g = grids[na - 1];
  LoopStartHeight = g.start_height;
  LoopStopHeight = g.stop_height;
  TotalHeightSteps = g.height_steps;
  return 0;
}

// ---- table walks (.cc:997-1302) on the host ------------------------------------------------
double Extrapolate(int Par, int index, double TotalHorizontalDistance, int AntennaNumber) {
  const std::vector<std::vector<float>>& t = host_table(AntennaNumber);
  const double x1 = t[1][index], x2 = t[1][index + 1];
  const double y1 = t[Par][index], y2 = t[Par][index + 1];
  const double m = (y2 - y1) / (x2 - x1);
  const double c = y1 - m * x1;
  return m * TotalHorizontalDistance + c;
}

double FindExtrapolationLimit(int index, double TotalHorizontalDistance, int AntennaNumber) {
  (void)TotalHorizontalDistance;  // unused by the reference (.cc:1026-1027 commented out)
  const std::vector<std::vector<float>>& t = host_table(AntennaNumber);
  const double x1 = t[1][index], x2 = t[1][index + 1];
  const double y1 = t[4][index], y2 = t[4][index + 1];
  const double m = (y1 - y2) / (x1 - x2);
  const double c = y1 - m * x1;
  return (90 - c) / m;
}

void FindClosestAirTxHeight(double ParValue, int& RStartIndex1, int& REndIndex1,
                            double& ClosestVal1, int& RStartIndex2, int& REndIndex2,
                            double& ClosestVal2, int AntennaNumber) {
  const airice::LkTable T = host_lk(host_table(AntennaNumber));
  int fl = 0;
  const airice::LkTxhBins b = airice::lk_closest_txh(T, ParValue, fl);
  RStartIndex1 = (int)b.s1;
  REndIndex1 = (int)b.e1;
  ClosestVal1 = b.c1;
  RStartIndex2 = (int)b.s2;
  REndIndex2 = (int)b.e2;
  ClosestVal2 = b.c2;
}

int FindClosestTHD(double ParValue, int StartIndex, int EndIndex, int& RStartIndex,
                   int& REndIndex, double& ClosestVal, int AntennaNumber) {
  const airice::LkTable T = host_lk(host_table(AntennaNumber));
  int fl = 0;
  airice::LkThdPair pr;  // host tables are not packed: the column path
  const airice::LkThdBins b = airice::lk_closest_thd(T, ParValue, StartIndex, EndIndex, fl, pr);
  RStartIndex = (int)b.s;
  REndIndex = (int)b.e;
  ClosestVal = b.c;
  return 0;
}

int GetParValues(double AntennaNumber, double AirTxHeight, double TotalHorizontalDistance,
                 double IceLayerHeight, double& AirTxHeight1, double Par1[10],
                 double& AirTxHeight2, double Par2[10]) {
  (void)IceLayerHeight;  // unused by the reference
  const std::vector<std::vector<float>>& cols = host_table((int)AntennaNumber);
  set_minmax(cols);
  const airice::LkTable T = host_lk(cols);
  int fl = 0;
  airice::lk_par_values(T, AirTxHeight, TotalHorizontalDistance, &AirTxHeight1, Par1,
                        &AirTxHeight2, Par2, fl);
  return 0;
}

bool TableLookup(double SrcHeightASL, double HorizontalDistanceToRx,
                 double RxDepthBelowIceBoundary, double IceLayerHeight, int TableIndex,
                 double& opticalPathLengthInIce, double& opticalPathLengthInAir,
                 double& geometricalPathLengthInIce, double& geometricalPathLengthInAir,
                 double& launchAngle, double& horizontalDistanceToIntersectionPoint,
                 double& transmissionCoefficientS, double& transmissionCoefficientP,
                 double& RecievedAngleInIce) {
  const std::vector<std::vector<float>>& cols = host_table(TableIndex);
  set_minmax(cols);
  const airice::LkTable T = host_lk(cols);
  double o[9];
  bool good = false;
  int fl = 0;
  // pi/180 exactly as the device's DevMedium::d2r (MultiRay pi, .cc:1410)
  if (airice::lk_query(T, SrcHeightASL / 100, HorizontalDistanceToRx / 100, pi / 180.0, o, &good,
                       fl)) {
    // the one-sided extrapolation case: the reference's minimizer fallback (.cc:1418-1420)
    const airice_medium m = medium();
    if (airice::lookup_fallback_one(&m, SrcHeightASL, HorizontalDistanceToRx,
                                    RxDepthBelowIceBoundary, IceLayerHeight, good, fl, o,
                                    &good) != AIRICE_OK)
      die("GetHorizontalDistanceToIntersectionPoint_Table fallback");
  }
  opticalPathLengthInIce = o[0];
  opticalPathLengthInAir = o[1];
  geometricalPathLengthInIce = o[2];
  geometricalPathLengthInAir = o[3];
  launchAngle = o[4];
  horizontalDistanceToIntersectionPoint = o[5];
  transmissionCoefficientS = o[6];
  transmissionCoefficientP = o[7];
  RecievedAngleInIce = o[8];
  return good;
}

bool GetHorizontalDistanceToIntersectionPoint_Table(
    double SrcHeightASL, double HorizontalDistanceToRx, double RxDepthBelowIceBoundary,
    double IceLayerHeight, int AntennaNumber, double& opticalPathLengthInIce,
    double& opticalPathLengthInAir, double& geometricalPathLengthInIce,
    double& geometricalPathLengthInAir, double& launchAngle,
    double& horizontalDistanceToIntersectionPoint, double& transmissionCoefficientS,
    double& transmissionCoefficientP, double& RecievedAngleInIce) {
  // antenna -> table remap over the caller's vectors (.cc:1348-1352)
  if (&AntennaDepths != nullptr && &AntennaTableAlreadyMade != nullptr) {
    for (int j = 0; j < (int)AntennaTableAlreadyMade.size(); j++)
      if (AntennaDepths[AntennaNumber] == AntennaDepths[AntennaTableAlreadyMade[j]])
        AntennaNumber = j;
  }
  return TableLookup(SrcHeightASL, HorizontalDistanceToRx, RxDepthBelowIceBoundary,
                     IceLayerHeight, AntennaNumber, opticalPathLengthInIce,
                     opticalPathLengthInAir, geometricalPathLengthInIce,
                     geometricalPathLengthInAir, launchAngle,
                     horizontalDistanceToIntersectionPoint, transmissionCoefficientS,
                     transmissionCoefficientP, RecievedAngleInIce);
}

void TableLookupBatch(const double* SrcHeightASL, const double* HorizontalDistanceToRx,
                      const double* RxDepthBelowIceBoundary, double IceLayerHeight, int TableIndex,
                      size_t n, double* out9, bool* ok) {
  const airice_medium m = medium();
  const std::vector<std::vector<float>>& cols = host_table(TableIndex);
  set_minmax(cols);
  if (n == 0) return;
  std::lock_guard<std::mutex> lock(g_mu);
  DevTable& dt = device_table(TableIndex);
  const size_t entries = dt.n;
  airice_lookup_table t;
  t.table = dt.dev;
  t.ld = entries;
  t.n_entries = entries;
  t.loop_stop_height = LoopStopHeight;  // globals of the last table made (.cc:1035-1039)
  t.height_step = HeightStepSize;
  t.total_height_steps = TotalHeightSteps;
  t.total_angle_steps = TotalAngleSteps;
  t.entries = nullptr;
  // the row records fix the row spans to the angle grid in force: re-pack when it changed
  if (dt.packed != nullptr && dt.packed_asteps != t.total_angle_steps) {
    (void)hipFree(dt.packed);
    dt.packed = nullptr;
  }
  if (dt.packed == nullptr) {
    if (t.total_angle_steps < 1 ||
        hipMalloc(&dt.packed, sizeof(float) * AIRICE_LOOKUP_PACK_FLOATS(entries, t.total_angle_steps)) != hipSuccess ||
        airice_lookup_pack(&t, dt.packed, AIRICE_LOOKUP_PACK_FLOATS(entries, t.total_angle_steps),
                           nullptr) != AIRICE_OK)
      die("airice_lookup_pack");
    dt.packed_asteps = t.total_angle_steps;
  }
  t.entries = dt.packed;
  // one device block: src | dist | depth | out (9 columns) | ok | flags
  void* mem = nullptr;
  if (hipMalloc(&mem, sizeof(double) * 12 * n + 2 * n) != hipSuccess) die("hipMalloc");
  double* d = static_cast<double*>(mem);
  if (hipMemcpy(d, SrcHeightASL, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d + n, HorizontalDistanceToRx, sizeof(double) * n, hipMemcpyHostToDevice) !=
          hipSuccess ||
      hipMemcpy(d + 2 * n, RxDepthBelowIceBoundary, sizeof(double) * n, hipMemcpyHostToDevice) !=
          hipSuccess)
    die("hipMemcpy");
  uint8_t* dok = reinterpret_cast<uint8_t*>(d + 12 * n);
  uint8_t* dfl = dok + n;
  if (airice_table_lookup_launch(&m, &t, d, d + n, d + 2 * n, IceLayerHeight, n, d + 3 * n, n, dok,
                                 dfl, nullptr) != AIRICE_OK)
    die("GetHorizontalDistanceToIntersectionPoint_Table");
  std::vector<double> soa(9 * n);
  std::vector<uint8_t> hok(n);
  if (hipMemcpy(soa.data(), d + 3 * n, sizeof(double) * 9 * n, hipMemcpyDeviceToHost) !=
          hipSuccess ||
      hipMemcpy(hok.data(), dok, n, hipMemcpyDeviceToHost) != hipSuccess)
    die("hipMemcpy");
  (void)hipFree(mem);
  for (size_t i = 0; i < n; ++i) {
    for (int c = 0; c < 9; ++c) out9[i * 9 + c] = soa[(size_t)c * n + i];
    ok[i] = hok[i] != 0;
  }
}

}  // namespace MultiRayAirIceRefraction
