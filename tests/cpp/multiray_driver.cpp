// CoREAS-style caller of the MultiRayAirIceRefraction:: drop-in (call sequence of
// RunMultiRayCode.C:29-59), linked against libairice.so.  Prints one JSON object.
#include <cmath>
#include <cstdio>
#include <vector>

#include "MultiRayAirIceRefraction.h"

std::vector<double> AntennaDepths;
std::vector<int> AntennaTableAlreadyMade;

static void arr(const char* name, const double* a, int n, bool last = false) {
  std::printf("\"%s\": [", name);
  for (int i = 0; i < n; ++i) std::printf("%.17g%s", a[i], i + 1 < n ? ", " : "");
  std::printf("]%s\n", last ? "" : ",");
}

int main() {
  namespace M = MultiRayAirIceRefraction;
  M::MakeAtmosphere();
  std::printf("{\n");
  double o[9];
  bool ok = M::GetHorizontalDistanceToIntersectionPoint(5000 * 100., 1000 * 100., -200 * 100.,
                                                        3000 * 100., o[0], o[1], o[2], o[3],
                                                        o[4], o[5], o[6], o[7], o[8]);
  std::printf("\"hdtip_ok\": %d,\n", ok ? 1 : 0);
  arr("hdtip", o, 9);
  double thR = 180 - (std::atan(1000. / (5000. - 3000. + 200.)) * (180.0 / M::pi));
  double d[20];
  M::Air2IceRayTracing(5000, 1000, 3000, -200, thR, d);
  arr("air2ice", d, 17);
  bool in_ice = true;
  M::GetRayTracingSolutions(170, 20000, 3000, -200, d, in_ice);
  arr("ray", d, 18);
  double fr[4] = {M::Refl_S(0.3, 3000), M::Trans_S(0.3, 3000), M::Refl_P(0.3, 3000),
                  M::Trans_P(0.3, 3000)};
  arr("fresnel", fr, 4);
  double nz[3] = {M::Getnz_air(3000), M::Getnz_air(50000), M::Getnz_ice(200)};
  arr("nz", nz, 3);
  // coarse grid through the reference's globals, two antennas with table dedupe
  HeightStepSize = 2000;
  AngleStepSize = 5;
  LoopStartAngle = 92;
  TotalAngleSteps = (int)std::floor((LoopStopAngle - LoopStartAngle) / AngleStepSize) + 1;
  AntennaDepths = {-200 * 100., -200 * 100., -100 * 100.};
  for (size_t i = 0; i < AntennaDepths.size(); ++i) {
    bool make = true;
    for (int j : AntennaTableAlreadyMade)
      if (AntennaDepths[i] == AntennaDepths[j]) make = false;
    if (make) {
      M::MakeRayTracingTable(AntennaDepths[i], 3000 * 100., (int)i);
      AntennaTableAlreadyMade.push_back((int)i);
    }
  }
  std::printf("\"tables\": %zu, \"rows\": %d, \"cols\": %d,\n", AllTableAllAntData.size(),
              TotalHeightSteps, TotalAngleSteps);
  std::printf("\"LoopStopHeight\": %.17g,\n", LoopStopHeight);
  std::vector<double> t1;
  for (int c = 0; c < 11; ++c) t1.push_back(AllTableAllAntData[1][c][123]);
  arr("table1_row123", t1.data(), 11);
  // table lookups through the reference entry (antenna 1 -> table 0, antenna 2 -> table 1)
  const double q[][2] = {{5000e2, 1000e2},  {20000e2, 15000e2}, {3500e2, 100e2},
                         {99999e2, 30000e2}, {200000e2, 1000e2}, {8000e2, 1e9},
                         {60000e2, 42000e2}, {3000e2, 10e2}};
  const int nq = sizeof(q) / sizeof(q[0]);
  std::printf("\"lookup\": [\n");
  for (int a = 0; a < 3; ++a)
    for (int i = 0; i < nq; ++i) {
      double r[10];
      bool okl = M::GetHorizontalDistanceToIntersectionPoint_Table(
          q[i][0], q[i][1], AntennaDepths[a], 3000 * 100., a, r[1], r[2], r[3], r[4], r[5], r[6],
          r[7], r[8], r[9]);
      r[0] = okl ? 1 : 0;
      std::printf("[%d, %.17g, %.17g, ", a, q[i][0], q[i][1]);
      for (int c = 0; c < 10; ++c) std::printf("%.17g%s", r[c], c < 9 ? ", " : "");
      std::printf("]%s\n", (a == 2 && i == nq - 1) ? "" : ",");
    }
  std::printf("],\n");
  std::printf("\"MaxAirTxHeight\": %.17g, \"MinAirTxHeight\": %.17g,\n", MaxAirTxHeight,
              MinAirTxHeight);
  for (int tbl = 0; tbl < 2; ++tbl) {
    std::printf("\"table%d\": [", tbl);
    for (int c = 0; c < 11; ++c) {
      std::printf("[");
      const std::vector<float>& col = AllTableAllAntData[tbl][c];
      for (size_t i = 0; i < col.size(); ++i)
        std::printf("%.9g%s", (double)col[i], i + 1 < col.size() ? ", " : "");
      std::printf("]%s", c < 10 ? ", " : "");
    }
    std::printf("]%s\n", tbl == 0 ? "," : "");
  }
  std::printf("}\n");
  return 0;
}
