// compat_common.h -- host pieces shared by the two C++ namespace drop-ins (compat_multiray.cpp,
// compat_rtf.cpp): reading Atmosphere.dat from the working directory and filling the reference's
// namespace data with its own stream semantics.  Both reference namespaces parse the file the
// same way: readATMpar (MultiRayAirIceRefraction.cc:24-71 == RayTracingFunctions.cc:4-49) and
// readnhFromFile (MultiRayAirIceRefraction.cc:73-147 == RayTracingFunctions.cc:51-124).
#pragma once
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "airice.h"

namespace airice_compat {

// Atmosphere.dat from the working directory, as the reference opens it, else $AIRICE_ATMOSPHERE.
// Missing file: abort with a message (the reference has no error channel; never fall back).
inline std::string atmosphere_text(const char* who) {
  const char* env = std::getenv("AIRICE_ATMOSPHERE");
  for (const char* path : {"Atmosphere.dat", env}) {
    if (path == nullptr) continue;
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) continue;
    std::ostringstream s;
    s << f.rdbuf();
    return s.str();
  }
  std::fprintf(stderr, "%s: Atmosphere.dat not found in the working directory or "
                       "$AIRICE_ATMOSPHERE\n", who);
  std::abort();
}

// readATMpar: the first four value rows, read with the reference's stream pattern (getline, then
// five >> reads from the following line); layer 4 copies layer 3, the top bound is 1500 km
inline void read_atm_par(const std::string& text, double ATMLAY[5], double abc[5][3]) {
  std::istringstream in(text);
  std::string line;
  double v[5] = {0, 0, 0, 0, 0};
  for (int row = 0; std::getline(in, line); ++row) {
    if (row < 4) in >> v[0] >> v[1] >> v[2] >> v[3] >> v[4];
    if (row == 0) for (int i = 0; i < 5; i++) ATMLAY[i] = v[i];
    if (row >= 1 && row <= 3) for (int i = 0; i < 5; i++) abc[i][row - 1] = v[i];
  }
  for (int k = 0; k < 3; k++) abc[4][k] = abc[3][k];
  ATMLAY[4] = 150000 * 100;
}

// readnhFromFile: (h, n) pairs from h > -1 m grouped into layers at the ATMLAY bounds, the
// duplicated last pair of the stream dropped; returns MaxLayers = layers + 1 (0: no profile)
inline int read_nh(const std::string& text, const double ATMLAY[5],
                   std::vector<std::vector<double>>& h_data,
                   std::vector<std::vector<double>>& nh_data,
                   std::vector<std::vector<double>>& lognh_data) {
  h_data.clear();
  nh_data.clear();
  lognh_data.clear();
  std::istringstream in(text);
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
  if (h_data.empty() || h_data.back().empty()) return 0;
  h_data.back().pop_back();
  nh_data.back().pop_back();
  lognh_data.back().pop_back();
  return (int)h_data.size() + 1;
}

// FillInAirRefractiveIndex (MultiRayAirIceRefraction.cc:193-213 == RayTracingFunctions.cc:149-170
// == pythonwrapper/AirIceRayTracing.cc:154-170) over a namespace's ATMLAY / abc: C_air from the
// scale heights, B_air chained for continuity from N0 (the natural cubic spline of the profile at
// 0 m, which the library's parse of the same file computes) with the namespace's A_air
inline void fill_air_index(const double ATMLAY[5], const double abc[5][3], double A_air,
                           double N0_spline, double C_air[5], double B_air[5]) {
  double N0 = 0;
  for (int il = 0; il < 5; il++) {
    const double hlow = ATMLAY[il] / 100;
    C_air[il] = 1.0 / (abc[il][2] / 100);
    if (il > 0) N0 = A_air + B_air[il - 1] * std::exp(-hlow * C_air[il - 1]);
    if (il == 0) N0 = N0_spline;
    B_air[il] = ((N0 - 1) / std::exp(-hlow * C_air[il]));
  }
}

// The medium a call runs on: the parse of the file (N0, profile size and top) with the namespace's
// current ATMLAY, B_air, C_air and MaxLayers -- the reference reads those at every call, so a
// caller's edits after MakeAtmosphere take effect
inline void apply_namespace(airice_medium& m, const double ATMLAY[5], const double B_air[5],
                            const double C_air[5], int MaxLayers) {
  for (int i = 0; i < 5; i++) {
    m.atmlay_cm[i] = ATMLAY[i];
    m.B_air[i] = B_air[i];
    m.C_air[i] = C_air[i];
  }
  m.max_layers = MaxLayers;
}

// flatten (MultiRayAirIceRefraction.cc:649-658 == RayTracingFunctions.cc:517-527)
inline std::vector<double> flatten(const std::vector<std::vector<double>>& v) {
  std::vector<double> r;
  for (const auto& s : v) r.insert(r.end(), s.begin(), s.end());
  return r;
}

}  // namespace airice_compat
