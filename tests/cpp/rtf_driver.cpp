// A RayTracingFunctions:: caller (the calls SingleRayAirIceRefraction.C and the RTF CLIs make),
// compiled against include/RayTracingFunctions.h and linked to libairice.so.  Prints one JSON
// object; tests/test_gpu_rtf.py compares it with the oracle.  Needs Atmosphere.dat in the cwd.
#include <cmath>
#include <cstdio>
#include <vector>

#include "RayTracingFunctions.h"

namespace R = RayTracingFunctions;

static void arr(const char* key, const double* v, int n, bool last = false) {
  std::printf("\"%s\": [", key);
  for (int i = 0; i < n; i++) std::printf("%s%.17g", i ? ", " : "", v[i]);
  std::printf("]%s\n", last ? "" : ",");
}

int main() {
  R::MakeAtmosphere();
  std::printf("{\n\"max_layers\": %d,\n", R::MaxLayers);
  arr("atmlay", R::ATMLAY, 5);
  arr("b_air", R::B_air, 5);
  arr("c_air", R::C_air, 5);
  std::printf("\"h_data_sizes\": [");
  for (size_t i = 0; i < R::h_data.size(); i++)
    std::printf("%s%zu", i ? ", " : "", R::h_data[i].size());
  std::printf("],\n\"h_top\": %.17g,\n", R::h_data.back().back());
  std::vector<double> flat = R::flatten(R::nh_data);
  std::printf("\"nh_flat\": %zu,\n", flat.size());
  const double nz[4] = {R::Getnz_air(0.0), R::Getnz_air(5000.0), R::Getnz_air(30000.0),
                        R::Getnz_ice(-100.0)};
  arr("nz", nz, 4);
  const double refl[2] = {R::Refl_S(0.5, 3000.0), R::Refl_P(0.5, 3000.0)};
  arr("refl", refl, 2);
  // SingleRayAirIceRefraction.C's first layer and ice leg (200 m antenna, 170 deg, 20 km Tx)
  double* hp = R::GetLayerHitPointPar(R::Getnz_air(20000.0), 8363.53902, 20000.0, 10.0, 1);
  arr("hit_air", hp, 4);
  delete[] hp;
  hp = R::GetLayerHitPointPar(1.0003, -200.0, 0.0, 9.9979, 0);
  arr("hit_ice", hp, 4);
  delete[] hp;
  double* ap = R::GetAirPropagationPar(170.0, 20000.0, 3000.0);
  arr("air_prop", ap, 4 * R::MaxLayers + 1);
  delete[] ap;
  double* ip = R::GetIcePropagationPar(9.9979, 3000.0, 200.0, 0.17365);
  arr("ice_prop", ip, 4);
  delete[] ip;
  R::MinforLAng_params mp = {20000.0, 3000.0, 200.0, 3000.0};
  R::fDnfR_params fp = {R::A_air, R::GetB_air(5000.0), -R::GetC_air(5000.0), 0.5};
  R::ftimeD_params tp = {R::A_ice, R::GetB_ice(100.0), -R::GetC_ice(100.0), R::spedc, 0.6, 0};
  const double scal[5] = {R::MinimizeforLaunchAngle(170.0, &mp), R::fDnfR(5000.0, &fp),
                          R::ftimeD(100.0, &tp),
                          R::GetRayOpticalPath(R::A_air, 3000.0, 8000.0, 0.4, 1),
                          R::GetRayPropagationTime(R::A_ice, 150.0, 0.0, 0.9, 0)};
  arr("scalars", scal, 5);
  // namespace data is read at every call: edit C_air of the 3217-8363 m layer, then undo it
  const double keep = R::C_air[1];
  R::C_air[1] = keep * 1.002;
  double* ep = R::GetAirPropagationPar(170.0, 20000.0, 3000.0);
  const double ed[3] = {ep[0] + ep[4] + ep[8], R::Getnz_air(5000.0), R::GetC_air(5000.0)};
  delete[] ep;
  R::C_air[1] = keep;
  arr("c_air_edit", ed, 3, true);
  std::printf("}\n");
  return 0;
}
