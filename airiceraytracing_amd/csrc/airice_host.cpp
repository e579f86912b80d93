// airice_host.cpp -- the host-only part of libairice.so: error reporting, GDAS Atmosphere.dat
// ingestion and the MakeRayTracingTable grid set-up.  No HIP here, so the same file also builds
// into the sanitizer harness (tests/cpp/asan_harness.cpp, `make asan`).
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "airice.h"
#include "airice_host.h"

namespace airice {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

double variant_pi(int variant) {
  // MultiRayAirIceRefraction.h:29 / RayTracingFunctions.h:26 vs pythonwrapper AirIceRayTracing.h:25
  return variant == AIRICE_VARIANT_PYWRAPPER ? 4.0 * std::atan(1.0) : 3.1415927;
}

// Natural cubic spline through (xs, ys) evaluated at x: second-derivative system
// solved by symmetric-tridiagonal LDL^T, then the cubic on the bracketing interval
// (the algorithm of gsl_interp_cspline, which the reference uses for n(h=0) only).
static double natural_spline_at(const std::vector<double>& xs, const std::vector<double>& ys,
                                 double x) {
  const size_t n = xs.size();
  const size_t m = n - 2;  // interior unknowns
  std::vector<double> c(n, 0.0), rhs(m), dg(m), od(m);
  for (size_t i = 0; i < m; ++i) {
    const double h0 = xs[i + 1] - xs[i], h1 = xs[i + 2] - xs[i + 1];
    const double g0 = (h0 != 0.0) ? 1.0 / h0 : 0.0;
    const double g1 = (h1 != 0.0) ? 1.0 / h1 : 0.0;
    od[i] = h1;
    dg[i] = 2.0 * (h1 + h0);
    rhs[i] = 3.0 * ((ys[i + 2] - ys[i + 1]) * g1 - (ys[i + 1] - ys[i]) * g0);
  }
  if (m == 1) {
    c[1] = rhs[0] / dg[0];
  } else {
    std::vector<double> piv(m), lo(m), z(m);
    piv[0] = dg[0];
    lo[0] = od[0] / piv[0];
    for (size_t i = 1; i + 1 < m; ++i) {
      piv[i] = dg[i] - od[i - 1] * lo[i - 1];
      lo[i] = od[i] / piv[i];
    }
    piv[m - 1] = dg[m - 1] - od[m - 2] * lo[m - 2];
    z[0] = rhs[0];
    for (size_t i = 1; i < m; ++i) z[i] = rhs[i] - lo[i - 1] * z[i - 1];
    for (size_t i = 0; i < m; ++i) z[i] = z[i] / piv[i];
    c[m] = z[m - 1];
    for (size_t k = m - 1; k-- > 0;) c[k + 1] = z[k] - lo[k] * c[k + 2];
  }
  size_t a = 0, b = n - 1;
  while (b > a + 1) {
    const size_t mid = (a + b) / 2;
    if (xs[mid] > x) b = mid; else a = mid;
  }
  const double dx = xs[a + 1] - xs[a];
  if (!(dx > 0.0)) return NAN;
  const double dy = ys[a + 1] - ys[a];
  const double t = x - xs[a];
  const double bi = (dy / dx) - dx * (c[a + 1] + 2.0 * c[a]) / 3.0;
  const double di = (c[a + 1] - c[a]) / (3.0 * dx);
  return ys[a] + t * (bi + t * (c[a] + t * di));
}

// GDAS Atmosphere.dat ingestion with the reference's stream semantics
// (readATMpar .cc:24-71, readnhFromFile .cc:73-147, FillInAirRefractiveIndex .cc:193-213).
int parse_gdas(const std::string& text, airice_medium* m) {
  std::memset(m, 0, sizeof(*m));
  m->A_air = 1.00;
  m->A_ice = 1.78;
  m->B_ice = -0.43;
  m->C_ice = 0.0132;
  m->A_const = 1.00;
  {
    std::istringstream in(text);
    std::string line;
    int row = 0;
    double v[5] = {0, 0, 0, 0, 0};
    while (std::getline(in, line)) {
      if (row < 4) in >> v[0] >> v[1] >> v[2] >> v[3] >> v[4];
      if (row == 0) for (int i = 0; i < 5; ++i) m->atmlay_cm[i] = v[i];
      if (row >= 1 && row <= 3) for (int i = 0; i < 5; ++i) m->abc[i][row - 1] = v[i];
      ++row;
    }
    for (int k = 0; k < 3; ++k) m->abc[4][k] = m->abc[3][k];
    m->atmlay_cm[4] = 150000 * 100;
  }
  std::vector<double> hs, ns;
  int groups = 0;
  {
    std::istringstream in(text);
    for (int i = 0; i < 5; ++i) in.ignore(256, '\n');
    std::string line;
    int layer = 0;
    double h = 0, nv = 0;
    while (std::getline(in, line)) {
      in >> h >> nv;  // at EOF the last pair is seen twice (removed below, .cc:137-140)
      if (h > -1) {
        hs.push_back(h);
        ns.push_back(nv);
        if (h * 100 >= m->atmlay_cm[layer < 4 ? layer : 4]) {
          if (layer > 0) ++groups;
          ++layer;
        }
      }
    }
    if (layer > 0) ++groups;
  }
  if (groups < 1 || hs.size() < 4) {
    set_error("atmosphere: no refractive-index profile found");
    return AIRICE_EIO;
  }
  hs.pop_back();
  ns.pop_back();
  m->max_layers = groups + 1;
  m->n_points = (int32_t)hs.size();
  m->h_top = hs.back();
  if (m->max_layers > kMaxParsedLayers) {
    set_error("atmosphere: %d layers exceed the 5 ATMLAY bounds", m->max_layers);
    return AIRICE_EINVAL;
  }
  m->N0 = natural_spline_at(hs, ns, 0.0);
  double N0 = 0;
  for (int il = 0; il < 5; ++il) {
    const double hlow = m->atmlay_cm[il] / 100;
    m->C_air[il] = 1.0 / (m->abc[il][2] / 100);
    if (il > 0) N0 = m->A_air + m->B_air[il - 1] * std::exp(-hlow * m->C_air[il - 1]);
    if (il == 0) N0 = m->N0;
    m->B_air[il] = ((N0 - 1) / std::exp(-hlow * m->C_air[il]));
  }
  return AIRICE_OK;
}

}  // namespace airice

using namespace airice;

extern "C" {

const char* airice_last_error(void) { return g_err; }
const char* airice_version(void) { return "airice-mi355x 0.1.0 (gfx950, fp64)"; }

int airice_atmosphere_parse(const char* text, size_t len, int variant, airice_medium* out) {
  if (text == nullptr || out == nullptr) {
    set_error("null argument");
    return AIRICE_EINVAL;
  }
  int rc = parse_gdas(std::string(text, len), out);
  if (rc == AIRICE_OK) out->pi = variant_pi(variant);
  return rc;
}

int airice_atmosphere_load(const char* path, int variant, airice_medium* out) {
  if (path == nullptr || out == nullptr) {
    set_error("null argument");
    return AIRICE_EINVAL;
  }
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) {
    set_error("cannot open atmosphere file '%s'", path);
    return AIRICE_EIO;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  return airice_atmosphere_parse(s.data(), s.size(), variant, out);
}

int airice_grid_init(airice_grid* g, double depth_cm, double ice_cm, double height_step,
                     double start_angle, double stop_angle, double angle_step) {
  if (g == nullptr || !(height_step > 0) || !(angle_step > 0) || !(stop_angle >= start_angle)) {
    set_error("invalid grid arguments");
    return AIRICE_EINVAL;
  }
  // MakeRayTracingTable (.cc:2021-2061)
  g->in_ice = depth_cm < 0 ? 1 : 0;
  g->depth_m = depth_cm / 100;
  g->ice_m = ice_cm / 100;
  g->start_height = 100000;
  g->stop_height = g->in_ice ? g->ice_m : g->ice_m + g->depth_m;
  g->height_step = height_step;
  // the reference's int conversions (.cc:2046, :15) of the step counts; counts beyond int range
  // (or NaN) would be undefined there and are rejected here
  const double hs = std::floor((g->start_height - g->stop_height) / height_step) + 1;
  const double as = std::floor((stop_angle - start_angle) / angle_step) + 1;
  if (!(hs >= 1 && hs <= 2147483647.0) || !(as >= 1 && as <= 2147483647.0)) {
    set_error("empty grid or step counts beyond int range (%g x %g)", hs, as);
    return AIRICE_EINVAL;
  }
  g->height_steps = (int32_t)hs;
  g->start_angle = start_angle;
  g->stop_angle = stop_angle;
  g->angle_step = angle_step;
  g->angle_steps = (int32_t)as;
  if (g->height_steps < 1 || g->angle_steps < 1) {
    set_error("empty grid");
    return AIRICE_EINVAL;
  }
  // The reference skips rows whose (unforced) AirTxHeight is not > 0 (.cc:2081-2082); heights
  // fall with the row index, so the kept rows are a prefix
  int32_t rows = g->height_steps;
  while (rows > 0 && !(g->start_height - g->height_step * (rows - 1) > 0)) --rows;
  g->table_rows = rows;
  return AIRICE_OK;
}

}  // extern "C"
