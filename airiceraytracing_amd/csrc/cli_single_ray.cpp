// SingleRayAirIceRefraction -- drop-in for the reference CLI (SingleRayAirIceRefraction.C, BASELINE
// cfg1): same arguments, stdout lines and RayPathinAirnIce.txt, with the ray traced and its path
// sampled on the GPU through libairice.so (airice_single_ray_host).
//
//   SingleRayAirIceRefraction <AntennaDepth m, >0 in ice> <launch deg> <TxHeight m> <IceHeight m>
//
// Reads Atmosphere.dat from the working directory like the reference (.C:33), falling back to
// $AIRICE_ATMOSPHERE.  The path file is written through one buffered stream (the reference
// flushes every line with std::endl); the text is the same default-precision ostream output.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <vector>

#include "airice.h"

static void usage() {
  std::cout << "Example run command: ./SingleRayAirIceRefraction 200 170 20000 3000" << std::endl;
  std::cout << "Here 200 is Antenna Depth in m, 170 is the ray launch angle (where is 0 vertically "
               "up) in deg, 20000 is the Tx Height in m and 3000 is Ice Layer Height in m"
            << std::endl;
}

int main(int argc, char** argv) {
  const auto t1 = std::chrono::high_resolution_clock::now();
  if (argc == 1) {
    std::cout << "No Extra Command Line Argument Passed Other Than Program Name" << std::endl;
    usage();
    return 0;
  }
  if (argc < 5) {
    std::cout << "More Arguments needed!" << std::endl;
    usage();
    return 0;
  }
  if (argc > 5) {
    std::cout << "More Arguments than needed!" << std::endl;
    usage();
    return 0;
  }
  std::cout << "Antenna Depth is set at " << std::atof(argv[1]) << " m, The Ray Launch Angle is set at "
            << std::atof(argv[2]) << " deg, Tx Height is set at " << std::atof(argv[3])
            << " m, Ice Layer Height is set as " << std::atof(argv[4]) << " m" << std::endl;

  airice_medium m;
  if (airice_atmosphere_load("Atmosphere.dat", AIRICE_VARIANT_MULTIRAY, &m) != AIRICE_OK) {
    const char* env = std::getenv("AIRICE_ATMOSPHERE");
    if (env == nullptr || airice_atmosphere_load(env, AIRICE_VARIANT_MULTIRAY, &m) != AIRICE_OK) {
      std::cerr << "SingleRayAirIceRefraction: cannot read Atmosphere.dat: " << airice_last_error()
                << std::endl;
      return 1;
    }
  }
  const double AntennaDepth = std::atof(argv[1]);
  double RayLaunchAngle = std::atof(argv[2]);
  double AirTxHeight = std::atof(argv[3]);
  const double IceLayerHeight = std::atof(argv[4]);

  if (AirTxHeight > m.h_top) {  // .C:40-45
    std::cout << "Tx Height is set higher than maximum available height for atmospheric refractive "
                 "index which is "
              << m.h_top << std::endl;
    AirTxHeight = m.h_top;
    std::cout << "Setting Tx Height to be the maximum available height" << std::endl;
  }
  if (RayLaunchAngle <= 90) {  // .C:47-51
    std::cout << "RayLaunchAngle has been set at " << RayLaunchAngle
              << " deg which is outside of the allowed range of 90 deg <RayLaunchAngle< 180 deg"
              << std::endl;
    RayLaunchAngle = 135;
    std::cout << "Setting RayLaunchAngle at" << RayLaunchAngle << std::endl;
  }
  std::ofstream aout("RayPathinAirnIce.txt");

  // the layer scans' messages (.C:60-86); the library repeats the scans for the trace
  const double* L = m.atmlay_cm;
  for (int il = m.max_layers; il > -1; il--) {
    if (AirTxHeight < L[il] / 100 && il >= 1 && AirTxHeight >= L[il - 1] / 100) {
      std::cout << "Tx Height is in this layer with a height range of " << L[il] / 100 << " m to "
                << L[il - 1] / 100 << " m and is at a height of " << AirTxHeight << " m" << std::endl;
      il = -100;
    }
  }
  for (int il = 0; il < m.max_layers; il++) {
    if (IceLayerHeight >= L[il] / 100 && IceLayerHeight < L[il + 1] / 100) {
      std::cout << "Ice Layer is in the layer with a height range of " << L[il] / 100 << " m to "
                << L[il + 1] / 100 << " m and is at a height of " << IceLayerHeight << " m"
                << std::endl;
      il = 100;
    }
  }

  airice_single_ray_info info;
  if (airice_single_ray_plan(&m, AntennaDepth, RayLaunchAngle, AirTxHeight, IceLayerHeight, &info) !=
      AIRICE_OK) {
    std::cerr << "SingleRayAirIceRefraction: " << airice_last_error() << std::endl;
    return 1;
  }
  const size_t n = (size_t)(info.n_air + info.n_ice);
  std::vector<double> x(n), z(n);
  double summary[AIRICE_SINGLE_RAY_FIELDS];
  if (airice_single_ray_host(&m, AntennaDepth, RayLaunchAngle, AirTxHeight, IceLayerHeight,
                             summary, x.data(), z.data(), n) != AIRICE_OK) {
    std::cerr << "SingleRayAirIceRefraction: " << airice_last_error() << std::endl;
    return 1;
  }
  std::cout << "Total horizontal distance travelled by the ray using Multiple Layer fitting is "
            << summary[0] << std::endl;
  std::cout << "Now treating the atmosphere refrative index profile as a single layer and fitting "
               "it and propogating the ray"
            << std::endl;
  for (size_t k = 0; k < n; ++k) aout << k << " " << x[k] << " " << z[k] << '\n';
  aout.close();

  const auto t2 = std::chrono::high_resolution_clock::now();
  long long ms = std::chrono::duration_cast<std::chrono::microseconds>(t2 - t1).count();
  ms = ms / 1000;
  std::cout << "total time taken by the script: " << ms << " ms" << std::endl;
  return 0;
}
