// Caller of the pythonwrapper library's C++ surface (pythonwrapper/AirIceRayTracing.h:23-146,
// TraceIceToAir.C:5) linked against libairice.so: namespace data, the ray layer, the three solve
// entry points on the queries of argv[1] (lines "depth ice txh dist", metres), FindFunctionRoot over
// MinimizeforLaunchAngle, the constant-index set-up of TraceIceToAir.C:27-29 and a B_air edit.
// Prints one JSON object that tests/test_gpu_pywrapper_cpp.py compares with the oracle.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "AirIceRayTracing.h"

namespace A = AirIceRayTracing;

static void arr(const char* name, const double* a, int n, const char* end = ",\n") {
  std::printf("\"%s\": [", name);
  for (int i = 0; i < n; ++i) std::printf("%.17g%s", a[i], i + 1 < n ? ", " : "");
  std::printf("]%s", end);
}

// thR of GetRayTracingSolution (AirIceRayTracing.cc:891-897)
static double straight_angle(double H, double D, double ice, double depth) {
  if (depth < 0) return 180 - (atan(D / (H - ice - depth)) * (180.0 / A::pi));
  return 180 - (atan(D / (H - (ice + depth))) * (180.0 / A::pi));
}

struct Q {
  double depth, ice, txh, dist;
};

// GetRayTracingSolution, Air2IceRayTracing, TraceIceToAir per query; prepare() runs before each
// query (TraceIceToAir re-reads the atmosphere file into the namespace, TraceIceToAir.C:25)
template <class Prep>
static void solves(const char* key, const std::vector<Q>& qs, Prep prepare) {
  std::printf("\"%s\": [\n", key);
  for (size_t i = 0; i < qs.size(); ++i) {
    const Q& q = qs[i];
    prepare();
    double o[8];
    const bool ok = A::GetRayTracingSolution(q.txh, q.dist, q.depth, q.ice, o[0], o[1], o[2], o[3],
                                             o[4], o[5], o[6], o[7]);
    double d[20];
    A::Air2IceRayTracing(q.txh, q.dist, q.ice, q.depth, straight_angle(q.txh, q.dist, q.ice, q.depth),
                         d);
    double t[10];
    TraceIceToAir(q.depth, q.ice, q.txh, q.dist, t);
    std::printf("[%d", ok ? 1 : 0);
    for (double v : o) std::printf(", %.17g", v);
    for (int k = 0; k < 15; ++k) std::printf(", %.17g", d[k]);
    for (double v : t) std::printf(", %.17g", v);
    std::printf("]%s\n", i + 1 < qs.size() ? "," : "");
  }
  std::printf("],\n");
}

int main(int argc, char** argv) {
  std::vector<Q> qs;
  if (argc > 1) {
    std::ifstream in(argv[1]);
    Q q;
    while (in >> q.depth >> q.ice >> q.txh >> q.dist) qs.push_back(q);
  }
  A::MakeAtmosphere("Atmosphere.dat");
  std::printf("{\n");
  std::printf("\"MaxLayers\": %d,\n", A::MaxLayers);
  arr("ATMLAY", A::ATMLAY, 5);
  arr("B_air", A::B_air, 5);
  arr("C_air", A::C_air, 5);
  std::printf("\"h_layers\": %zu, \"h_points\": %zu,\n", A::h_data.size(),
              A::flatten(A::h_data).size());
  const double nz[6] = {A::Getnz_air(3000), A::Getnz_air(50000), A::Getnz_ice(-200),
                        A::GetB_air(12000), A::GetC_air(12000), A::Getnz_air(-7000)};
  arr("nz", nz, 6);
  const double fr[4] = {A::Refl_S(0.3, 3000), A::Trans_S(0.3, 3000), A::Refl_P(0.3, 3000),
                        A::Trans_P(0.3, 3000)};
  arr("fresnel", fr, 4);
  // the ray layer (.cc:356-857)
  {
    A::fDnfR_params p{A::A_ice, A::GetB_ice(-150), -A::GetC_ice(-150), 1.5};
    A::ftimeD_params q{A::A_ice, A::GetB_ice(-150), -A::GetC_ice(-150), A::spedc, 1.5, 0};
    const double v[3] = {A::fDnfR(-150, &p), A::ftimeD(-150, &q), A::fpathD(-150, &q)};
    arr("f_ice", v, 3);
    A::fDnfR_params pa{A::A_air, A::GetB_air(5000), -A::GetC_air(5000), 0.8};
    A::ftimeD_params qa{A::A_air, A::GetB_air(5000), -A::GetC_air(5000), A::spedc, 0.8, 1};
    const double va[3] = {A::fDnfR(5000, &pa), A::ftimeD(5000, &qa), A::fpathD(5000, &qa)};
    arr("f_air", va, 3);
    const double w[6] = {A::GetRayHorizontalPath(A::A_air, 3000, 9000, 0.7, 1),
                         A::GetRayPropagationTime(A::A_air, 3000, 9000, 0.7, 1),
                         A::GetRayGeometricPath(A::A_air, 3000, 9000, 0.7, 1),
                         A::GetRayHorizontalPath(A::A_ice, -200, 0, 1.2, 0),
                         A::GetRayPropagationTime(A::A_ice, -200, 0, 1.2, 0),
                         A::GetRayGeometricPath(A::A_ice, -200, 0, 1.2, 0)};
    arr("paths", w, 6);
    double* h = A::GetLayerHitPointPar(A::Getnz_air(9000), 3000, 9000, 35.0, 1);
    arr("hit_air", h, 5);
    delete[] h;
    double* a = A::GetAirPropagationPar(160.0, 20000.0, 3000.0);
    arr("air_prop", a, 5 * A::MaxLayers + 2);
    delete[] a;
    double* b = A::GetIcePropagationPar(30.0, 3000, 200, 0.9);
    arr("ice_prop", b, 5);
    delete[] b;
    double ml[3];
    for (int k = 0; k < 3; ++k) {
      A::MinforLAng_params mp{20000.0, 3000.0, 200.0, 1000.0 + 9000.0 * k};
      ml[k] = A::MinimizeforLaunchAngle(150.0 + 5 * k, &mp);
    }
    arr("min_launch", ml, 3);
  }
  solves("solves", qs, [] {});
  // the reference's own search: FindFunctionRoot(MinimizeforLaunchAngle, bisection, 1e-9, 40) over
  // the bracket [thR - 16, thR] of the first queries (no probe needed there), ray layer on the GPU
  {
    std::printf("\"find_root\": [");
    const size_t nr = qs.size() < 4 ? qs.size() : 4;
    for (size_t i = 0; i < nr; ++i) {
      const Q& q = qs[i];
      const double thR = straight_angle(q.txh, q.dist, q.ice, q.depth);
      A::MinforLAng_params mp{q.txh, q.ice, -q.depth, q.dist};
      gsl_function F;
      F.function = &A::MinimizeforLaunchAngle;
      F.params = &mp;
      const double lo = thR - 16 < 90.001 ? 90.001 : thR - 16;
      const double r1 = A::FindFunctionRoot(F, lo, thR, gsl_root_fsolver_bisection, 1e-9, 40);
      const double r2 = A::FindFunctionRoot(F, lo, thR, gsl_root_fsolver_brent, 1e-9, 40);
      std::printf("[%.17g, %.17g, %.17g, %.17g]%s", lo, thR, r1, r2, i + 1 < nr ? ", " : "");
    }
    std::printf("],\n");
  }
  // an edit of the namespace data is read by the next call (here: B_air of the Tx layer)
  {
    const double keep = A::B_air[1];
    std::vector<Q> one(qs.begin(), qs.begin() + (qs.size() < 3 ? qs.size() : 3));
    solves("solves_b_air_edit", one, [keep] { A::B_air[1] = keep * 1.001; });
  }
  // constant refractive index (TraceIceToAir.C:27-29, commented out in the reference)
  {
    A::A_const = A::Getnz_air(3000);
    A::UseConstantRefractiveIndex = true;
    A::A_air = A::A_const;
    const double c[4] = {A::Getnz_air(5000), A::GetB_air(5000), A::GetC_air(5000), A::A_const};
    arr("const_nz", c, 4);
    std::vector<Q> one(qs.begin(), qs.begin() + (qs.size() < 3 ? qs.size() : 3));
    solves("solves_const", one, [] {});
    A::UseConstantRefractiveIndex = false;
    A::A_air = 1.00;
    A::A_const = 1.00;
    A::MakeAtmosphere("Atmosphere.dat");
  }
  const double after[2] = {A::B_air[1], A::Getnz_air(3000)};
  arr("restored", after, 2, "\n");
  std::printf("}\n");
  return 0;
}
