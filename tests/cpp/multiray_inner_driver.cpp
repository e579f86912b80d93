// Caller of the MultiRayAirIceRefraction:: inner API (MultiRayAirIceRefraction.h:33-204 of the
// reference): namespace data, the ray layer, the table walks, the exported _Table and its
// antenna remap, linked against libairice.so.  Prints one JSON object that
// tests/test_gpu_compat.py compares with the oracle.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "MultiRayAirIceRefraction.h"

std::vector<double> AntennaDepths;
std::vector<int> AntennaTableAlreadyMade;

namespace M = MultiRayAirIceRefraction;

static void arr(const char* name, const double* a, int n) {
  std::printf("\"%s\": [", name);
  for (int i = 0; i < n; ++i) std::printf("%.17g%s", a[i], i + 1 < n ? ", " : "");
  std::printf("],\n");
}

int main() {
  M::MakeAtmosphere();
  std::printf("{\n");
  // namespace data (.h:33-84)
  std::printf("\"MaxLayers\": %d,\n", M::MaxLayers);
  arr("ATMLAY", M::ATMLAY, 5);
  arr("B_air", M::B_air, 5);
  arr("C_air", M::C_air, 5);
  double abcf[15];
  for (int i = 0; i < 5; ++i)
    for (int k = 0; k < 3; ++k) abcf[i * 3 + k] = M::abc[i][k];
  arr("abc", abcf, 15);
  const std::vector<double> hflat = M::flatten(M::h_data), nflat = M::flatten(M::nh_data);
  std::printf("\"h_layers\": %zu, \"h_points\": %zu,\n", M::h_data.size(), hflat.size());
  const double hn[4] = {hflat.front(), hflat.back(), nflat.front(), nflat.back()};
  arr("h_n_ends", hn, 4);
  // the ray layer (.cc:377-917): ice and air forms
  {
    M::fDnfR_params p{M::A_ice, M::GetB_ice(-150), -M::GetC_ice(-150), 1.5};
    M::ftimeD_params q{M::A_ice, M::GetB_ice(-150), -M::GetC_ice(-150), M::spedc, 1.5, 0};
    const double v[3] = {M::fDnfR(-150, &p), M::ftimeD(-150, &q), M::fpathD(-150, &q)};
    arr("f_ice", v, 3);
    M::fDnfR_params pa{M::A_air, M::GetB_air(5000), -M::GetC_air(5000), 0.8};
    M::ftimeD_params qa{M::A_air, M::GetB_air(5000), -M::GetC_air(5000), M::spedc, 0.8, 1};
    const double va[3] = {M::fDnfR(5000, &pa), M::ftimeD(5000, &qa), M::fpathD(5000, &qa)};
    arr("f_air", va, 3);
  }
  {
    const double v[6] = {M::GetRayHorizontalPath(M::A_air, 3000, 9000, 0.7, 1),
                         M::GetRayPropagationTime(M::A_air, 3000, 9000, 0.7, 1),
                         M::GetRayGeometricPath(M::A_air, 3000, 9000, 0.7, 1),
                         M::GetRayHorizontalPath(M::A_ice, -200, 0, 1.2, 0),
                         M::GetRayPropagationTime(M::A_ice, -200, 0, 1.2, 0),
                         M::GetRayGeometricPath(M::A_ice, -200, 0, 1.2, 0)};
    arr("paths", v, 6);
  }
  {
    double* a = M::GetLayerHitPointPar(M::Getnz_air(9000), 3000, 9000, 35.0, 1);
    arr("hit_air", a, 5);
    delete[] a;
    double* b = M::GetLayerHitPointPar(M::Getnz_air(3000), -200, 0, 35.0, 0);
    arr("hit_ice", b, 5);
    delete[] b;
  }
  const double launches[][2] = {{160.0, 20000.0}, {120.0, 90000.0}, {95.0, 5000.0}};
  for (int k = 0; k < 3; ++k) {
    double* a = M::GetAirPropagationPar(launches[k][0], launches[k][1], 3000);
    std::string nm = "air_prop" + std::to_string(k);
    arr(nm.c_str(), a, 5 * M::MaxLayers + 2);
    delete[] a;
  }
  {
    double* a = M::GetIcePropagationPar(30.0, 3000, -200, 0.9);
    arr("ice_prop", a, 5);
    delete[] a;
  }
  {
    double v[3];
    for (int k = 0; k < 3; ++k) {
      M::MinforLAng_params p{20000.0, 3000.0, -200.0, 1000.0 + 9000.0 * k};
      v[k] = M::MinimizeforLaunchAngle(150.0 + 5 * k, &p);
    }
    arr("min_launch", v, 3);
  }
  // the ice model is read at every call (.h:75-77): change A_ice, then restore it
  {
    double v[2];
    M::A_ice = 1.775;
    v[0] = M::Getnz_ice(-100);
    double* a = M::GetIcePropagationPar(30.0, 3000, -200, 0.9);
    v[1] = a[0];
    delete[] a;
    M::A_ice = M::A_ice_def;
    arr("a_ice_1775", v, 2);
  }
  // the air model is namespace data read at every call (.h:56-61): an edit of B_air[1] (the
  // 3217-8363 m layer) after MakeAtmosphere changes the next solve, ray and n(z), then is undone
  {
    const double keep = M::B_air[1];
    M::B_air[1] = keep * 1.001;
    double d[20], rr[20];
    const double thR = 180 - (std::atan(1000.0 / 2200.0) * (180.0 / M::pi));
    M::Air2IceRayTracing(5000.0, 1000.0, 3000.0, -200.0, thR, d);
    arr("air2ice_b_air_edit", d, 17);
    bool in_ice = true;
    M::GetRayTracingSolutions(170.0, 20000.0, 3000.0, -200.0, rr, in_ice);
    arr("ray_b_air_edit", rr, 18);
    const double nz[2] = {M::Getnz_air(5000), M::GetB_air(5000)};
    arr("nz_b_air_edit", nz, 2);
    M::B_air[1] = keep;
  }
  // coarse table through the reference's globals, two antennas with table dedupe
  HeightStepSize = 2000;
  AngleStepSize = 5;
  LoopStartAngle = 92;
  TotalAngleSteps = (int)std::floor((LoopStopAngle - LoopStartAngle) / AngleStepSize) + 1;
  AntennaDepths = {-200 * 100., -100 * 100., -200 * 100.};
  for (size_t i = 0; i < AntennaDepths.size(); ++i) {
    bool make = true;
    for (int j : AntennaTableAlreadyMade)
      if (AntennaDepths[i] == AntennaDepths[j]) make = false;
    if (make) {
      M::MakeRayTracingTable(AntennaDepths[i], 3000 * 100., (int)i);
      AntennaTableAlreadyMade.push_back((int)i);
    }
  }
  // MakeRayTracingTables (one launch) against the per-antenna tables just made, plus an
  // antenna in the air made both ways
  {
    const size_t before = AllTableAllAntData.size();
    M::MakeRayTracingTables({-200 * 100., -100 * 100., 50 * 100.}, 3000 * 100.);
    M::MakeRayTracingTable(50 * 100., 3000 * 100., 3);
    auto bits_equal = [](const std::vector<std::vector<float>>& x,
                         const std::vector<std::vector<float>>& y) {  // NaN entries included
      if (x.size() != y.size()) return 0;
      for (size_t c = 0; c < x.size(); ++c)
        if (x[c].size() != y[c].size() ||
            std::memcmp(x[c].data(), y[c].data(), sizeof(float) * x[c].size()) != 0)
          return 0;
      return 1;
    };
    const int same[3] = {bits_equal(AllTableAllAntData[before], AllTableAllAntData[0]),
                         bits_equal(AllTableAllAntData[before + 1], AllTableAllAntData[1]),
                         bits_equal(AllTableAllAntData[before + 2], AllTableAllAntData[before + 3])};
    std::printf("\"multi_tables_equal\": [%d, %d, %d],\n", same[0], same[1], same[2]);
    AllTableAllAntData.resize(before);  // drop them again: the remap below sees tables 0 and 1
    M::MakeRayTracingTable(-100 * 100., 3000 * 100., 1);  // restores the last-table globals
    AllTableAllAntData.pop_back();
  }
  std::printf("\"grid\": [%.17g, %.17g, %d, %d],\n", LoopStopHeight, HeightStepSize,
              TotalHeightSteps, TotalAngleSteps);
  // table walks on table 0 (.cc:997-1302)
  const double heights[] = {99999.0, 51234.5, 23000.0, 3000.0, 4321.0, 8000.0};
  std::printf("\"closest_txh\": [");
  for (int k = 0; k < 6; ++k) {
    int s1, e1, s2, e2;
    double c1, c2;
    M::FindClosestAirTxHeight(heights[k], s1, e1, c1, s2, e2, c2, 0);
    std::printf("[%d, %d, %.17g, %d, %d, %.17g]%s", s1, e1, c1, s2, e2, c2, k < 5 ? ", " : "");
  }
  std::printf("],\n");
  std::printf("\"closest_thd\": [");
  for (int k = 0; k < 6; ++k) {
    int s1, e1, s2, e2, rs, re;
    double c1, c2, c;
    M::FindClosestAirTxHeight(heights[k], s1, e1, c1, s2, e2, c2, 0);
    M::FindClosestTHD(1500.0 * (k + 1), s1, e1, rs, re, c, 0);
    std::printf("[%d, %d, %.17g]%s", rs, re, c, k < 5 ? ", " : "");
  }
  std::printf("],\n");
  std::printf("\"par_values\": [");
  for (int k = 0; k < 6; ++k) {
    double h1, h2, p1[10], p2[10];
    M::GetParValues(0, heights[k], 1500.0 * (k + 1), 3000, h1, p1, h2, p2);
    std::printf("[%.17g, ", h1);
    for (int i = 0; i < 10; ++i) std::printf("%.17g, ", p1[i]);
    std::printf("%.17g, ", h2);
    for (int i = 0; i < 10; ++i) std::printf("%.17g%s", p2[i], i < 9 ? ", " : "");
    std::printf("]%s", k < 5 ? ", " : "");
  }
  std::printf("],\n");
  std::printf("\"MaxMinAirTxHeight\": [%.17g, %.17g],\n", MaxAirTxHeight, MinAirTxHeight);
  const double ex[4] = {M::Extrapolate(2, 40, 12000.0, 0), M::Extrapolate(7, 41, 3000.0, 1),
                        M::FindExtrapolationLimit(40, 12000.0, 0),
                        M::FindExtrapolationLimit(41, 0.0, 1)};
  arr("extrapolate", ex, 4);
  // the exported _Table (antenna 2 -> table 0 by depth) against the batched GPU lookup
  const double q[][2] = {{5000e2, 1000e2},  {20000e2, 15000e2}, {3500e2, 100e2},
                         {99999e2, 30000e2}, {200000e2, 1000e2}, {8000e2, 1e9},
                         {60000e2, 42000e2}, {3000e2, 10e2},     {41000e2, 39000e2}};
  const int nq = sizeof(q) / sizeof(q[0]);
  std::printf("\"table_scalar_vs_batch\": [\n");
  for (int a = 0; a < 3; ++a) {
    const int table = a == 1 ? 1 : 0;
    std::vector<double> src(nq), dst(nq), dep(nq, AntennaDepths[a]), out9(9 * nq);
    bool okb[16];
    for (int i = 0; i < nq; ++i) {
      src[i] = q[i][0];
      dst[i] = q[i][1];
    }
    M::TableLookupBatch(src.data(), dst.data(), dep.data(), 3000 * 100., table, nq, out9.data(),
                        okb);
    for (int i = 0; i < nq; ++i) {
      double r[9];
      const bool ok = M::GetHorizontalDistanceToIntersectionPoint_Table(
          q[i][0], q[i][1], AntennaDepths[a], 3000 * 100., a, r[0], r[1], r[2], r[3], r[4], r[5],
          r[6], r[7], r[8]);
      int same = ok == okb[i];
      for (int c = 0; c < 9; ++c) {
        const double g = out9[i * 9 + c];
        if (!(r[c] == g || (std::isnan(r[c]) && std::isnan(g)))) same = 0;
      }
      std::printf("[%d, %d, %d, %d]%s\n", a, i, ok ? 1 : 0, same,
                  (a == 2 && i == nq - 1) ? "" : ",");
    }
  }
  std::printf("],\n");
  std::printf("\"table0\": [");
  for (int c = 0; c < 11; ++c) {
    std::printf("[");
    const std::vector<float>& col = AllTableAllAntData[0][c];
    for (size_t i = 0; i < col.size(); ++i)
      std::printf("%.9g%s", (double)col[i], i + 1 < col.size() ? ", " : "");
    std::printf("]%s", c < 10 ? ", " : "");
  }
  std::printf("],\n");
  std::printf("\"table1_col1\": [");
  const std::vector<float>& t1 = AllTableAllAntData[1][1];
  for (size_t i = 0; i < t1.size(); ++i)
    std::printf("%.9g%s", (double)t1[i], i + 1 < t1.size() ? ", " : "");
  std::printf("],\n");
  std::printf("\"table1_col\": [");
  for (int c = 0; c < 11; ++c) {
    const std::vector<float>& col = AllTableAllAntData[1][c];
    std::printf("[%.9g, %.9g]%s", (double)col[41], (double)col[42], c < 10 ? ", " : "");
  }
  std::printf("]\n}\n");
  return 0;
}
