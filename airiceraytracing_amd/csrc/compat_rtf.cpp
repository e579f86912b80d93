// compat_rtf.cpp -- RayTracingFunctions:: C++ surface over the C-ABI
// (include/RayTracingFunctions.h).  Keeps the reference's globals, call semantics and heap-array
// outputs; every ray quantity is evaluated on the GPU (airice_rtf_eval, airice_rtf.hip).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "RayTracingFunctions.h"
#include "airice.h"

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

// Atmosphere.dat from the working directory, as the reference opens it (.cc:6, 55), else
// $AIRICE_ATMOSPHERE
std::string atmosphere_text() {
  const char* env = std::getenv("AIRICE_ATMOSPHERE");
  for (const char* path : {"Atmosphere.dat", env}) {
    if (path == nullptr) continue;
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) continue;
    std::ostringstream s;
    s << f.rdbuf();
    return s.str();
  }
  std::fprintf(stderr, "RayTracingFunctions: Atmosphere.dat not found in the working directory "
                       "or $AIRICE_ATMOSPHERE\n");
  std::abort();
}

const airice_medium& medium() {
  if (!g_have_medium) R::MakeAtmosphere();
  return g_medium;
}

// one GPU evaluation of a RayTracingFunctions quantity
void rtf(int op, std::initializer_list<double> args, double* out, size_t n_out) {
  const std::vector<double> a(args);
  if (airice_rtf_eval(&medium(), op, a.data(), a.size(), out, n_out) != AIRICE_OK)
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

// readATMpar (.cc:4-49): the first four value rows, read with the reference's stream pattern
// (getline, then five >> reads from the following line); layer 4 copies layer 3, top 1500 km
int readATMpar() {
  std::istringstream in(atmosphere_text());
  std::string line;
  double v[5] = {0, 0, 0, 0, 0};
  for (int row = 0; std::getline(in, line); ++row) {
    if (row < 4) in >> v[0] >> v[1] >> v[2] >> v[3] >> v[4];
    if (row == 0) for (int i = 0; i < 5; i++) ATMLAY[i] = v[i];
    if (row >= 1 && row <= 3) for (int i = 0; i < 5; i++) abc[i][row - 1] = v[i];
  }
  for (int k = 0; k < 3; k++) abc[4][k] = abc[3][k];
  ATMLAY[4] = 150000 * 100;
  return 0;
}

// readnhFromFile (.cc:51-124): (h, n) pairs from h > -1 m, grouped into layers at the ATMLAY
// bounds, the duplicated last pair of the stream dropped; MaxLayers = layers + 1
int readnhFromFile() {
  nh_data.clear();
  lognh_data.clear();
  h_data.clear();
  std::istringstream in(atmosphere_text());
  for (int i = 0; i < 5; i++) in.ignore(256, '\n');
  std::string line;
  int layer = 0;
  double h = 0, n = 0;
  std::vector<double> th, tn, tl;
  while (std::getline(in, line)) {
    in >> h >> n;
    if (h > -1) {
      th.push_back(h);
      tn.push_back(n);
      tl.push_back(std::log(n - 1));
      if (h * 100 >= ATMLAY[layer < 4 ? layer : 4]) {  // (a profile above 1500 km would index
                                                     //  past ATMLAY in the reference)
        if (layer > 0) {
          h_data.push_back(th);
          nh_data.push_back(tn);
          lognh_data.push_back(tl);
          th.clear();
          tn.clear();
          tl.clear();
        }
        layer++;
      }
    }
  }
  if (layer > 0) {
    h_data.push_back(th);
    nh_data.push_back(tn);
    lognh_data.push_back(tl);
  }
  if (h_data.empty() || h_data.back().empty()) {
    std::fprintf(stderr, "RayTracingFunctions: no refractive-index profile in Atmosphere.dat\n");
    std::abort();
  }
  h_data.back().pop_back();
  nh_data.back().pop_back();
  lognh_data.back().pop_back();
  MaxLayers = (int)h_data.size() + 1;
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
  for (int i = 0; i < 5; i++) {
    C_air[i] = g_medium.C_air[i];
    B_air[i] = g_medium.B_air[i];
  }
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
double Getnz_ice(double z) { return airice_nz_ice(&medium(), z); }
double GetB_air(double z) {
  medium();
  return B_air[layer_of(z)];
}
double GetC_air(double z) {
  medium();
  return C_air[layer_of(z)];
}
double Getnz_air(double z) { return airice_nz_air(&medium(), z); }

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
  std::vector<double> r;
  for (const auto& s : v) r.insert(r.end(), s.begin(), s.end());
  return r;
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
