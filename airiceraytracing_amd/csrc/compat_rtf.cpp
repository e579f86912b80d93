// compat_rtf.cpp -- RayTracingFunctions:: C++ surface over the C-ABI
// (include/RayTracingFunctions.h).  Keeps the reference's globals, call semantics and heap-array
// outputs; every ray quantity is evaluated on the GPU (airice_rtf_eval, airice_rtf.hip).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "RayTracingFunctions.h"
#include "airice.h"
#include "compat_common.h"

namespace RayTracingFunctions {

std::vector<std::vector<double>> nh_data;
std::vector<std::vector<double>> lognh_data;
std::vector<std::vector<double>> h_data;
double ATMLAY[5];
double abc[5][3];
double C_air[5];
double B_air[5];
int MaxLayers = 0;

}  // namespace RayTracingFunctions

namespace {

namespace R = RayTracingFunctions;

std::mutex g_mu;
airice_medium g_medium;
bool g_have_medium = false;

[[noreturn]] void die(const char* what) {
  std::fprintf(stderr, "RayTracingFunctions: %s failed: %s\n", what, airice_last_error());
  std::abort();  // the reference has no error channel; fail loudly, never fall back
}

std::string atmosphere_text() { return airice_compat::atmosphere_text("RayTracingFunctions"); }

// The medium of the next call: the parse of the file with the namespace's current ATMLAY, B_air,
// C_air and MaxLayers (the reference reads them at every call, so edits take effect)
airice_medium medium() {
  if (!g_have_medium) R::MakeAtmosphere();
  airice_medium m = g_medium;
  airice_compat::apply_namespace(m, R::ATMLAY, R::B_air, R::C_air, R::MaxLayers);
  return m;
}

// one GPU evaluation of a RayTracingFunctions quantity
void rtf(int op, std::initializer_list<double> args, double* out, size_t n_out) {
  const std::vector<double> a(args);
  const airice_medium m = medium();
  if (airice_rtf_eval(&m, op, a.data(), a.size(), out, n_out) != AIRICE_OK)
    die("airice_rtf_eval");
}

double rtf1(int op, std::initializer_list<double> args) {
  double r = 0;
  rtf(op, args, &r, 1);
  return r;
}

int layer_of(double z) {  // GetB_air / GetC_air scan over the globals (.cc:172-213)
  const double zabs = std::fabs(z);
  int which = 0;
  for (int il = 0; il < R::MaxLayers - 1; il++) {
    if (zabs < R::ATMLAY[il + 1] / 100 && zabs >= R::ATMLAY[il] / 100) {
      which = il;
      break;
    }
  }
  if (zabs >= R::ATMLAY[R::MaxLayers - 1] / 100) which = R::MaxLayers - 1;
  return which;
}

}  // namespace

namespace RayTracingFunctions {

// readATMpar (.cc:4-49)
int readATMpar() {
  airice_compat::read_atm_par(atmosphere_text(), ATMLAY, abc);
  return 0;
}

// readnhFromFile (.cc:51-124): MaxLayers = layers + 1
int readnhFromFile() {
  MaxLayers = airice_compat::read_nh(atmosphere_text(), ATMLAY, h_data, nh_data, lognh_data);
  if (MaxLayers == 0) {
    std::fprintf(stderr, "RayTracingFunctions: no refractive-index profile in Atmosphere.dat\n");
    std::abort();
  }
  return 0;
}

// FillInAirRefractiveIndex (.cc:149-170): N0 from the natural cubic spline of the profile at 0 m,
// then B_air chained for continuity -- the library's parse of the same file does exactly this
int FillInAirRefractiveIndex() {
  const std::string text = atmosphere_text();
  if (airice_atmosphere_parse(text.data(), text.size(), AIRICE_VARIANT_MULTIRAY, &g_medium) !=
      AIRICE_OK)
    die("FillInAirRefractiveIndex");
  g_have_medium = true;
  airice_compat::fill_air_index(ATMLAY, abc, A_air, g_medium.N0, C_air, B_air);
  return 0;
}

// MakeAtmosphere (.cc:733-754)
int MakeAtmosphere() {
  std::lock_guard<std::mutex> lock(g_mu);
  readATMpar();
  readnhFromFile();
  FillInAirRefractiveIndex();
  return 0;
}

double GetB_ice(double) { return -0.43; }  // .cc:126-133
double GetC_ice(double) { return 0.0132; } // .cc:135-142
double Getnz_ice(double z) {
  const airice_medium m = medium();
  return airice_nz_ice(&m, z);
}
double GetB_air(double z) {
  medium();
  return B_air[layer_of(z)];
}
double GetC_air(double z) {
  medium();
  return C_air[layer_of(z)];
}
double Getnz_air(double z) {
  const airice_medium m = medium();
  return airice_nz_air(&m, z);
}

// Refl_S / Refl_P (.cc:222-255): power reflectances, NaN -> 1
double Refl_S(double thetai, double IceLayerHeight) {
  const double n1 = Getnz_air(IceLayerHeight), n2 = Getnz_ice(0);
  const double s = (n1 / n2) * std::sin(thetai);
  const double sq = std::sqrt(1 - s * s);
  const double num = n1 * std::cos(thetai) - n2 * sq, den = n1 * std::cos(thetai) + n2 * sq;
  const double r = (num * num) / (den * den);
  return std::isnan(r) ? 1 : r;
}
double Refl_P(double thetai, double IceLayerHeight) {
  const double n1 = Getnz_air(IceLayerHeight), n2 = Getnz_ice(0);
  const double s = (n1 / n2) * std::sin(thetai);
  const double sq = std::sqrt(1 - s * s);
  const double num = n1 * sq - n2 * std::cos(thetai), den = n1 * sq + n2 * std::cos(thetai);
  const double r = (num * num) / (den * den);
  return std::isnan(r) ? 1 : r;
}

double fDnfR(double x, void* params) {
  const fDnfR_params* p = static_cast<const fDnfR_params*>(params);
  return rtf1(AIRICE_RTF_FDNFR, {x, p->a, p->b, p->c, p->l});
}

double ftimeD(double x, void* params) {
  const ftimeD_params* p = static_cast<const ftimeD_params*>(params);
  return rtf1(AIRICE_RTF_FTIMED, {x, p->a, p->b, p->c, p->speedc, p->l, (double)p->airorice});
}

double GetRayOpticalPath(double A, double RxDepth, double TxDepth, double Lvalue, int AirOrIce) {
  return rtf1(AIRICE_RTF_OPTICAL_PATH, {A, RxDepth, TxDepth, Lvalue, (double)AirOrIce});
}

double GetRayPropagationTime(double A, double RxDepth, double TxDepth, double Lvalue,
                             int AirOrIce) {
  return rtf1(AIRICE_RTF_PROPAGATION_TIME, {A, RxDepth, TxDepth, Lvalue, (double)AirOrIce});
}

double* GetLayerHitPointPar(double n_layer1, double RxDepth, double TxDepth, double IncidentAng,
                            int AirOrIce) {
  double* out = new double[4];
  rtf(AIRICE_RTF_HIT_POINT, {n_layer1, RxDepth, TxDepth, IncidentAng, (double)AirOrIce}, out, 4);
  return out;
}

std::vector<double> flatten(const std::vector<std::vector<double>>& v) {  // .cc:517-527
  return airice_compat::flatten(v);
}

double* GetAirPropagationPar(double LaunchAngle, double AirTxHeight, double IceLayerHeight) {
  const int n = 4 * medium().max_layers + 1;
  double* out = new double[n];
  rtf(AIRICE_RTF_AIR_PROPAGATION, {LaunchAngle, AirTxHeight, IceLayerHeight}, out, n);
  return out;
}

double* GetIcePropagationPar(double IncidentAngleonIce, double IceLayerHeight, double AntennaDepth,
                             double Lvalue) {
  double* out = new double[4];
  rtf(AIRICE_RTF_ICE_PROPAGATION, {IncidentAngleonIce, IceLayerHeight, AntennaDepth, Lvalue}, out,
      4);
  return out;
}

double MinimizeforLaunchAngle(double x, void* params) {
  const MinforLAng_params* p = static_cast<const MinforLAng_params*>(params);
  return rtf1(AIRICE_RTF_MIN_LAUNCH,
              {x, p->airtxheight, p->icelayerheight, p->antennadepth, p->horizontaldistance});
}

}  // namespace RayTracingFunctions
