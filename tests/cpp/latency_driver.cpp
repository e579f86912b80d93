// Per-call latency of the scalar drop-in entry points, called one query at a time with host
// arguments the way CoREAS (RunMultiRayCode.C:29-59) and TraceIceToAir.py call them.  Linked
// against libairice.so; run by bench.py (scalar_latency_us) from a directory holding
// Atmosphere.dat.  Prints one JSON line: per entry point the mean and median microseconds of
// 400 calls after 20 warm-up calls, on cfg3-distributed queries (mt19937_64, seed 12345).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "MultiRayAirIceRefraction.h"
#include "RayTracingFunctions.h"
#include "airice.h"

std::vector<double> AntennaDepths;
std::vector<int> AntennaTableAlreadyMade;

namespace {

struct Q {
  double txh, dist, depth;
};

std::string timeit(const char* name, const std::vector<Q>& qs,
                   const std::function<void(const Q&)>& call, bool last = false) {
  const int warm = 20, reps = (int)qs.size();
  for (int i = 0; i < warm; ++i) call(qs[i % qs.size()]);
  std::vector<double> us(reps);
  for (int i = 0; i < reps; ++i) {
    auto t0 = std::chrono::steady_clock::now();
    call(qs[i]);
    auto t1 = std::chrono::steady_clock::now();
    us[i] = std::chrono::duration<double, std::micro>(t1 - t0).count();
  }
  double mean = 0;
  for (double u : us) mean += u;
  mean /= reps;
  std::sort(us.begin(), us.end());
  char buf[256];
  std::snprintf(buf, sizeof(buf), "\"%s\": {\"mean\": %.3f, \"median\": %.3f, \"calls\": %d}%s",
                name, mean, us[reps / 2], reps, last ? "" : ", ");
  return buf;
}

}  // namespace

int main() {
  namespace M = MultiRayAirIceRefraction;
  M::MakeAtmosphere();
  // cfg2 grid through the reference's globals, one antenna 200 m deep
  HeightStepSize = 20;
  AngleStepSize = 0.5;
  LoopStartAngle = 92;
  TotalAngleSteps = (int)std::floor((LoopStopAngle - LoopStartAngle) / AngleStepSize) + 1;
  AntennaDepths = {-200 * 100.};
  M::MakeRayTracingTable(AntennaDepths[0], 3000 * 100., 0);
  AntennaTableAlreadyMade.push_back(0);

  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> uh(3001, 100000), ud(0, 50000), uz(0, 300);
  std::vector<Q> qs(400);
  for (Q& q : qs) {
    q.txh = uh(rng);
    q.dist = ud(rng);
    q.depth = -uz(rng);
  }
  double o[20];
  double sink = 0;
  std::string s = "{";
  s += timeit("GetHorizontalDistanceToIntersectionPoint", qs, [&](const Q& q) {
    M::GetHorizontalDistanceToIntersectionPoint(q.txh * 100, q.dist * 100, -200 * 100.,
                                                3000 * 100., o[0], o[1], o[2], o[3], o[4], o[5],
                                                o[6], o[7], o[8]);
    sink += o[5];
  });
  s += timeit("GetHorizontalDistanceToIntersectionPoint_Table", qs, [&](const Q& q) {
    M::GetHorizontalDistanceToIntersectionPoint_Table(q.txh * 100, q.dist * 100, -200 * 100.,
                                                      3000 * 100., 0, o[0], o[1], o[2], o[3],
                                                      o[4], o[5], o[6], o[7], o[8]);
    sink += o[5];
  });
  s += timeit("Air2IceRayTracing", qs, [&](const Q& q) {
    const double thr =
        180 - std::atan(q.dist / (q.txh - 3000 - q.depth)) * (180.0 / M::pi);
    M::Air2IceRayTracing(q.txh, q.dist, 3000, q.depth, thr, o);
    sink += o[0];
  });
  s += timeit("GetRayTracingSolutions", qs, [&](const Q& q) {
    bool in_ice = true;
    M::GetRayTracingSolutions(92 + std::fmod(q.dist, 88.0), q.txh, 3000, -200, o, in_ice);
    sink += o[1];
  });
  s += timeit("RayTracingFunctions::GetAirPropagationPar", qs, [&](const Q& q) {
    double* r = RayTracingFunctions::GetAirPropagationPar(92 + std::fmod(q.dist, 88.0), q.txh,
                                                          3000);
    sink += r[0];
    delete[] r;
  });
  s += timeit("Py_TraceIceToAir", qs, [&](const Q& q) {
    double a[10];
    Py_TraceIceToAir(q.depth, 3000, q.txh < 20000 ? q.txh : 20000, q.dist * 0.6, a);
    sink += a[0];
  }, true);
  s += "}";
  std::printf("%s\n", s.c_str());
  std::fprintf(stderr, "checksum %g\n", sink);
  return 0;
}
