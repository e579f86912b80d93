// compat_pywrapper.cpp -- AirIceRayTracing:: C++ surface (the reference's pythonwrapper library,
// pythonwrapper/AirIceRayTracing.h:23-146 / AirIceRayTracing.cc / TraceIceToAir.C) over the C-ABI
// (include/AirIceRayTracing.h).  Numerics are AIRICE_VARIANT_PYWRAPPER (pi = 4*atan(1)).  Solves
// and the ray layer run on the GPU, one query per call through the current device's pinned scalar
// slot; the atmosphere readers, the n(z) layer scans and the Fresnel coefficients are host code
// as in the reference.
#include <hip/hip_runtime.h>
#include <sys/stat.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <iostream>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "AirIceRayTracing.h"
#include "airice.h"
#include "airice_internal.h"
#include "compat_common.h"

// ---- namespace data (.h:29-72): one shared copy, read by every call -------------------------
namespace AirIceRayTracing {
std::vector<std::vector<double>> nh_data;
std::vector<std::vector<double>> lognh_data;
std::vector<std::vector<double>> h_data;
double ATMLAY[5];
double abc[5][3];
double C_air[5];
double B_air[5];
int MaxLayers = 0;
bool UseConstantRefractiveIndex = false;
double A_air = 1.00;
double A_const = 1.00;
}  // namespace AirIceRayTracing

namespace {

namespace PY = AirIceRayTracing;

[[noreturn]] void die(const char* what) {
  std::fprintf(stderr, "AirIceRayTracing: %s failed: %s\n", what, airice_last_error());
  std::abort();  // the reference has no error channel; fail loudly, never fall back
}

// The last atmosphere file read: its text and its parse (N0 = the natural cubic spline of its
// profile at 0 m, .cc:871-873 + :164).  Re-read when the file's identity, size or mtime changes.
struct AtmFile {
  std::string path;
  dev_t dev = 0;
  ino_t ino = 0;
  off_t size = -1;
  struct timespec mtime = {0, 0};
  std::string text;
  airice_medium parsed;
  double atmlay[5];  // readATMpar of the text (ATMLAY, abc), kept with it
  double abc[5][3];
  bool valid = false;
  unsigned long long gen = 0;  // parse number
};
std::recursive_mutex g_mu;
AtmFile g_atm;
bool g_made = false;  // MakeAtmosphere has filled the namespace data at least once

bool same_file(const AtmFile& a, const std::string& path, const struct stat& st) {
  return a.valid && a.path == path && a.dev == st.st_dev && a.ino == st.st_ino &&
         a.size == st.st_size && a.mtime.tv_sec == st.st_mtim.tv_sec &&
         a.mtime.tv_nsec == st.st_mtim.tv_nsec;
}

// The named file, else $AIRICE_ATMOSPHERE (this repo's convention for a missing working-directory
// file); parsed once while unchanged.
const AtmFile& atmosphere_file(const std::string& name) {
  const char* env = std::getenv("AIRICE_ATMOSPHERE");
  for (const char* p : {name.c_str(), env}) {
    if (p == nullptr) continue;
    struct stat st;
    if (stat(p, &st) != 0) continue;
    if (same_file(g_atm, p, st)) return g_atm;
    AtmFile f;
    f.path = p;
    f.dev = st.st_dev;
    f.ino = st.st_ino;
    f.size = st.st_size;
    f.mtime = st.st_mtim;
    std::ifstream in(p, std::ios::binary);
    if (!in.is_open()) continue;
    std::ostringstream s;
    s << in.rdbuf();
    f.text = s.str();
    if (airice_atmosphere_parse(f.text.data(), f.text.size(), AIRICE_VARIANT_PYWRAPPER,
                                &f.parsed) != AIRICE_OK)
      die("MakeAtmosphere");
    airice_compat::read_atm_par(f.text, f.atmlay, f.abc);
    f.valid = true;
    f.gen = g_atm.gen + 1;
    g_atm = std::move(f);
    return g_atm;
  }
  std::fprintf(stderr, "AirIceRayTracing: atmosphere file '%s' not found (nor $AIRICE_ATMOSPHERE)\n",
               name.c_str());
  std::abort();
}

// FillInAirRefractiveIndex (.cc:154-170) over the namespace data and the current A_air
void fill_air_index(double N0_spline) {
  airice_compat::fill_air_index(PY::ATMLAY, PY::abc, PY::A_air, N0_spline, PY::C_air, PY::B_air);
}

// The medium of the next call: the namespace data as it is now (the reference reads it at every
// call), with the spline-derived fields of the last file read.
airice_medium medium() {
  std::lock_guard<std::recursive_mutex> lock(g_mu);
  if (!g_made) PY::MakeAtmosphere("Atmosphere.dat");
  airice_medium m = g_atm.parsed;
  airice_compat::apply_namespace(m, PY::ATMLAY, PY::B_air, PY::C_air, PY::MaxLayers);
  m.A_air = PY::A_air;
  m.A_const = PY::A_const;
  m.constant_air_index = PY::UseConstantRefractiveIndex ? 1 : 0;
  m.A_ice = PY::A_ice;
  m.B_ice = -0.43;  // GetB_ice (.cc:131-137)
  m.C_ice = 0.0132; // GetC_ice (.cc:140-146)
  m.pi = PY::pi;
  return m;
}

// one GPU evaluation of a ray-layer quantity with the pythonwrapper's numerics
void ray_op(int op, std::initializer_list<double> args, double* out, size_t n_out) {
  const airice_medium m = medium();
  const std::vector<double> a(args);
  if (airice_rtf_eval_variant(&m, AIRICE_VARIANT_PYWRAPPER, op, a.data(), a.size(), out, n_out) !=
      AIRICE_OK)
    die("ray layer");
}

double ray_op1(int op, std::initializer_list<double> args) {
  double r = 0;
  ray_op(op, args, &r, 1);
  return r;
}

int layer_of(double zabs) {  // GetB_air / GetC_air layer scan (.cc:180-189)
  int which = 0;
  for (int il = 0; il < PY::MaxLayers - 1; il++) {
    if (zabs < PY::ATMLAY[il + 1] / 100 && zabs >= PY::ATMLAY[il] / 100) {
      which = il;
      break;
    }
  }
  if (PY::MaxLayers >= 1 && zabs >= PY::ATMLAY[PY::MaxLayers - 1] / 100) which = PY::MaxLayers - 1;
  return which;
}

// one launch-angle solve through the scalar slot: dummy[0..14] (.cc:1070-1084), status bits
void solve_one(const airice_medium& m, double H, double D, double ice, double depth,
               const double* straight_angle, double dummy[AIRICE_PYSOLVE_FIELDS]) {
  if (airice::scalar_on_host()) {  // one query: on the host (airice_scalar_mode)
    const double in[4] = {H, D, depth, straight_angle != nullptr ? *straight_angle : 0.0};
    if (airice::solve_query_host(&m, AIRICE_VARIANT_PYWRAPPER, ice, in, straight_angle != nullptr,
                                 dummy, nullptr) != AIRICE_OK)
      die("Air2IceRayTracing");
    return;
  }
  airice::ScalarCall call;
  if (!call.ok()) die("Air2IceRayTracing");
  airice::ScalarSlot& s = call.slot();
  s.h[0] = H;
  s.h[1] = D;
  s.h[2] = depth;
  s.h[3] = straight_angle != nullptr ? *straight_angle : 0.0;
  call.arm(s.h, straight_angle != nullptr ? 4 : 3);
  if (airice_solve_launch(&m, AIRICE_VARIANT_PYWRAPPER, ice, s.d, s.d + 1, s.d + 2,
                          straight_angle != nullptr ? s.d + 3 : nullptr, 1, s.d + 4, 1, nullptr,
                          s.st) != AIRICE_OK ||
      call.sync() != AIRICE_OK)
    die("Air2IceRayTracing");
  std::memcpy(dummy, s.h + 4, sizeof(double) * AIRICE_PYSOLVE_FIELDS);
}

}  // namespace

namespace AirIceRayTracing {

// ---- atmosphere (.cc:4-128, 154-170, 860-881) ----------------------------------------------
int readATMpar(std::string atmosFileName) {
  std::lock_guard<std::recursive_mutex> lock(g_mu);
  airice_compat::read_atm_par(atmosphere_file(atmosFileName).text, ATMLAY, abc);
  return 0;
}

int readnhFromFile(std::string atmosFileName) {
  std::lock_guard<std::recursive_mutex> lock(g_mu);
  MaxLayers =
      airice_compat::read_nh(atmosphere_file(atmosFileName).text, ATMLAY, h_data, nh_data, lognh_data);
  if (MaxLayers == 0) {
    std::fprintf(stderr, "AirIceRayTracing: no refractive-index profile in '%s'\n",
                 atmosFileName.c_str());
    std::abort();  // the reference indexes an empty vector here (.cc:119)
  }
  return 0;
}

int FillInAirRefractiveIndex() {
  std::lock_guard<std::recursive_mutex> lock(g_mu);
  if (!g_atm.valid) {  // the reference evaluates a spline that was never set up (.cc:164)
    std::fprintf(stderr, "AirIceRayTracing: FillInAirRefractiveIndex before MakeAtmosphere\n");
    std::abort();
  }
  fill_air_index(g_atm.parsed.N0);
  return 0;
}

std::vector<double> flatten(const std::vector<std::vector<double>>& v) {  // .cc:628-637
  return airice_compat::flatten(v);
}

int MakeAtmosphere(std::string atmosFileName) {
  std::lock_guard<std::recursive_mutex> lock(g_mu);
  const AtmFile& f = atmosphere_file(atmosFileName);
  // readATMpar's values for this file (parsed once per file version: TraceIceToAir calls this on
  // every query, TraceIceToAir.C:25)
  std::memcpy(ATMLAY, f.atmlay, sizeof(ATMLAY));
  std::memcpy(abc, f.abc, sizeof(abc));
  // the profile vectors are re-read when the file changed or their shape differs; their values
  // feed only the spline, whose N0 comes from the same file
  static unsigned long long filled_gen = 0;
  const int layers = f.parsed.max_layers - 1;
  if (!g_made || filled_gen != f.gen || (int)h_data.size() != layers ||
      (int)nh_data.size() != layers || (int)lognh_data.size() != layers)
    readnhFromFile(atmosFileName);
  else
    MaxLayers = f.parsed.max_layers;
  filled_gen = f.gen;
  fill_air_index(f.parsed.N0);
  g_made = true;
  return 0;
}

// ---- n(z) (.cc:131-239) --------------------------------------------------------------------
double GetB_ice(double) { return -0.43; }
double GetC_ice(double) { return 0.0132; }
double Getnz_ice(double z) {
  z = std::fabs(z);
  return A_ice + GetB_ice(z) * std::exp(-GetC_ice(z) * z);
}

double GetB_air(double z) {
  medium();
  if (UseConstantRefractiveIndex) return 0;
  return B_air[layer_of(std::fabs(z))];
}

double GetC_air(double z) {
  medium();
  if (UseConstantRefractiveIndex) return 1e-9;
  return C_air[layer_of(std::fabs(z))];
}

double Getnz_air(double z) {
  const double zabs = std::fabs(z);
  if (UseConstantRefractiveIndex) return A_const;
  return A_air + GetB_air(zabs) * std::exp(-GetC_air(zabs) * zabs);
}

// ---- Fresnel amplitude coefficients (.cc:242-312) ------------------------------------------
static void fresnel(double thetai, double ice, double& rS, double& tS, double& rP, double& tP) {
  const double n1 = Getnz_air(ice), n2 = Getnz_ice(0);
  const double a = (n1 / n2) * std::sin(thetai);
  const double sq = std::sqrt(1 - a * a);  // pow(x, 2) == x * x
  double num = n1 * std::cos(thetai) - n2 * sq, den = n1 * std::cos(thetai) + n2 * sq;
  rS = num / den;
  tS = 1 + (num / den);
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

// ---- the ray layer (.cc:356-857) on the GPU ------------------------------------------------
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
  ray_op(AIRICE_MR_HIT_POINT, {n_layer1, RxDepth, TxDepth, IncidentAng, (double)AirOrIce}, out, 5);
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

// ---- one-query solves ----------------------------------------------------------------------
void Air2IceRayTracing(double AirTxHeight, double HorizontalDistance, double IceLayerHeight,
                       double AntennaDepth, double StraightAngle, double dummy[20]) {
  solve_one(medium(), AirTxHeight, HorizontalDistance, IceLayerHeight, AntennaDepth,
            &StraightAngle, dummy);
}

bool GetRayTracingSolution(double SrcHeightASL, double HorizontalDistanceToRx,
                           double RxDepthBelowIceBoundary, double IceLayerHeight,
                           double& opticalPathLengthInIce, double& opticalPathLengthInAir,
                           double& geometricalPathLengthInIce, double& geometricalPathLengthInAir,
                           double& launchAngle, double& horizontalDistanceToIntersectionPoint,
                           double& AngleOfIncidenceOnIce, double& RecievedAngleInIce) {
  const double D = HorizontalDistanceToRx;
  double dm[AIRICE_PYSOLVE_FIELDS];
  // thR (.cc:891-897) is formed by the kernel from the same expression
  solve_one(medium(), SrcHeightASL, D, IceLayerHeight, RxDepthBelowIceBoundary, nullptr, dm);
  opticalPathLengthInIce = dm[5];
  opticalPathLengthInAir = dm[6];
  geometricalPathLengthInIce = dm[14];
  geometricalPathLengthInAir = dm[13];
  launchAngle = dm[10];
  horizontalDistanceToIntersectionPoint = dm[2];
  AngleOfIncidenceOnIce = dm[11];
  RecievedAngleInIce = dm[12];
  bool CheckSolution = false;  // .cc:912-921
  if ((std::fabs(dm[1] - D) / D < 0.01 && D <= 100) || (std::fabs(dm[1] - D) < 1 && D > 100))
    CheckSolution = true;
  if (dm[1] < 0) CheckSolution = false;
  return CheckSolution;
}

}  // namespace AirIceRayTracing

// ---- TraceIceToAir.C:5-79 ------------------------------------------------------------------
void TraceIceToAir(double AntennaDepth, double IceLayerHeight, double AirTxHeight,
                   double HorizontalDistance, double ArrayParameters[10]) {
  airice_medium m;
  {
    std::lock_guard<std::recursive_mutex> lock(g_mu);
    AirIceRayTracing::MakeAtmosphere("Atmosphere.dat");  // TraceIceToAir.C:25
    m = medium();
  }
  // GetRayTracingSolution + the launch/receive swap + ArrayParameters (TraceIceToAir.C:27-68):
  // one launch of the batch trace path with n = 1
  if (airice::scalar_on_host()) {  // one query: on the host (airice_scalar_mode)
    const double in[4] = {AntennaDepth, IceLayerHeight, AirTxHeight, HorizontalDistance};
    if (airice::trace_query_host(&m, in, ArrayParameters) != AIRICE_OK) die("TraceIceToAir");
  } else {
    airice::ScalarCall call;
    if (!call.ok()) die("TraceIceToAir");
    airice::ScalarSlot& s = call.slot();
    s.h[0] = AntennaDepth;
    s.h[1] = IceLayerHeight;
    s.h[2] = AirTxHeight;
    s.h[3] = HorizontalDistance;
    call.arm(s.h, 4);
    if (airice_trace_ice_to_air_launch(&m, s.d, s.d + 1, s.d + 2, s.d + 3, 1, s.d + 4, s.st) !=
            AIRICE_OK ||
        call.sync() != AIRICE_OK)
      die("TraceIceToAir");
    std::memcpy(ArrayParameters, s.h + 4, sizeof(double) * 10);
  }
  static const bool verbose = [] {
    const char* v = std::getenv("AIRICE_VERBOSE");
    return v != nullptr && std::strcmp(v, "1") == 0;
  }();
  if (verbose) {  // TraceIceToAir.C:35-55
    const double* a = ArrayParameters;
    if (a[0] != -1000 || a[9] != -1000) {
      std::cout << " We have a solution!!!" << std::endl;
      std::cout << "AirTxHeight: " << a[0] << std::endl;
      std::cout << "HorizontalDistance: " << a[1] << std::endl;
      std::cout << "geometricalPathLengthInIce: " << a[2] << std::endl;
      std::cout << "geometricalPathLengthInAir: " << a[3] << std::endl;
      std::cout << "launchAngle: " << a[4] << std::endl;
      std::cout << "RecievedAngle: " << a[5] << std::endl;
      std::cout << "horidist2interpnt: " << a[6] << std::endl;
      std::cout << "AngleOfIncidenceOnIce: " << a[7] << std::endl;
    } else {
      std::cout << " We do NOT have a solution!!!" << std::endl;
    }
  }
}

extern "C" void Py_TraceIceToAir(double AntennaDepth, double IceLayerHeight, double AirTxHeight,
                                 double HorizontalDistance, double ArrayParameters[10]) {
  TraceIceToAir(AntennaDepth, IceLayerHeight, AirTxHeight, HorizontalDistance, ArrayParameters);
}
