// Air2IceRayTracing -- drop-in for the reference CLI (Air2IceRayTracing.C): same arguments and
// stdout lines; the launch-angle search (bracket, probe, GSL-Brent root of
// RayTracingFunctions::MinimizeforLaunchAngle) and the air results run on the GPU as one
// airice_rtf_eval(AIRICE_RTF_AIR2ICE) call, the ice results as GetIcePropagationPar
// (AIRICE_RTF_ICE_PROPAGATION), through libairice.so.
//
//   Air2IceRayTracing <TxHeight m> <horizontal distance m> <IceHeight m> <AntennaDepth m, > 0 in ice>
//
// Reads Atmosphere.dat from the working directory like the reference (RayTracingFunctions::
// MakeAtmosphere), falling back to $AIRICE_ATMOSPHERE.  StoreRayPath is false in the reference
// (Air2IceRayTracing.C:56), so no path file is written here either.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "airice.h"

static void usage() {
  std::cout << "Example run command: ./Air2IceRayTracing 5000 1000 3000 200" << std::endl;
  std::cout << "Here 5000 m is Tx Height in air in m, 1000 is the horizontal distance btw Tx in "
               "air and Rx in ice in m, 3000 is Ice Layer Height in m and 200 is the Antenna "
               "Depth in ice in m"
            << std::endl;
}

int main(int argc, char** argv) {
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
  std::cout << "Tx Height in air is set at " << std::atof(argv[1])
            << " m, the horizontal distance btw Tx in air and Rx in ice is set at "
            << std::atof(argv[2]) << " m, Ice Layer Height is set at " << std::atof(argv[3])
            << " m, Antenna Depth is set at " << std::atof(argv[4]) << " m" << std::endl;
  if (std::atof(argv[1]) < std::atof(argv[3])) {
    std::cout << "WARNING: AirTxHeight is less than IceLayerHeight." << std::endl;
    std::cout << "Please set the AirTxHeight to be above the IceLayerHeight" << std::endl;
    return 0;
  }
  const auto t1b = std::chrono::high_resolution_clock::now();
  const auto t1b_atm = std::chrono::high_resolution_clock::now();
  airice_medium m;
  if (airice_atmosphere_load("Atmosphere.dat", AIRICE_VARIANT_MULTIRAY, &m) != AIRICE_OK) {
    const char* env = std::getenv("AIRICE_ATMOSPHERE");
    if (env == nullptr || airice_atmosphere_load(env, AIRICE_VARIANT_MULTIRAY, &m) != AIRICE_OK) {
      std::cerr << "Air2IceRayTracing: cannot read Atmosphere.dat: " << airice_last_error()
                << std::endl;
      return 1;
    }
  }
  const auto t2b_atm = std::chrono::high_resolution_clock::now();
  const double AirTxHeight = std::atof(argv[1]);
  const double HorizontalDistance = std::atof(argv[2]);
  const double IceLayerHeight = std::atof(argv[3]);
  const double AntennaDepth = std::atof(argv[4]);

  const auto t1b_air = std::chrono::high_resolution_clock::now();
  const double args[4] = {AirTxHeight, HorizontalDistance, IceLayerHeight, AntennaDepth};
  double r[AIRICE_RTF_AIR2ICE_FIELDS];
  if (airice_rtf_eval(&m, AIRICE_RTF_AIR2ICE, args, 4, r, AIRICE_RTF_AIR2ICE_FIELDS) !=
      AIRICE_OK) {
    std::cerr << "Air2IceRayTracing: " << airice_last_error() << std::endl;
    return 1;
  }
  const auto t2b_air = std::chrono::high_resolution_clock::now();
  std::cout << "Launch Angle search range is:  Startangle " << r[0] << " ,Endangle " << r[1]
            << std::endl;
  std::cout << " " << std::endl;
  std::cout << "***********Results for Air************" << std::endl;
  std::cout << "TotalHorizontalDistanceinAir " << r[3] << " m" << std::endl;
  std::cout << "IncidentAngleonIce " << r[4] << " deg" << std::endl;
  std::cout << "LvalueAir for " << r[5] << std::endl;
  std::cout << "PropagationTimeAir " << r[6] << " ns" << std::endl;

  const auto t1b_ice = std::chrono::high_resolution_clock::now();
  const double iargs[4] = {r[4], IceLayerHeight, AntennaDepth, r[5]};
  double ice[4];
  if (airice_rtf_eval(&m, AIRICE_RTF_ICE_PROPAGATION, iargs, 4, ice, 4) != AIRICE_OK) {
    std::cerr << "Air2IceRayTracing: " << airice_last_error() << std::endl;
    return 1;
  }
  const double PropagationTimeIce = ice[3] * 1e9;
  const auto t2b_ice = std::chrono::high_resolution_clock::now();
  std::cout << " " << std::endl;
  std::cout << "***********Results for Ice************" << std::endl;
  std::cout << "TotalHorizontalDistanceinIce " << ice[0] << " m" << std::endl;
  std::cout << "IncidentAngleonAntenna " << ice[1] << " deg" << std::endl;
  std::cout << "LvalueIce " << r[5] << std::endl;
  std::cout << "PropagationTimeIce " << PropagationTimeIce << " ns" << std::endl;
  std::cout << " " << std::endl;
  std::cout << "***********Results for Ice + Air************" << std::endl;
  std::cout << "TotalHorizontalDistance " << ice[0] + r[3] << " m" << std::endl;
  std::cout << "TotalPropagationTime " << PropagationTimeIce + r[6] << " ns" << std::endl;

  using std::chrono::duration_cast;
  using us = std::chrono::microseconds;
  using ns = std::chrono::nanoseconds;
  const auto t2b = std::chrono::high_resolution_clock::now();
  std::cout << "total time taken by the script to do solution calcuation: "
            << duration_cast<us>(t2b - t1b).count() / 1000 << " ms" << std::endl;
  std::cout << "total time taken by the script to do solution calcuation for Ice: "
            << duration_cast<ns>(t2b_ice - t1b_ice).count() << " ns" << std::endl;
  std::cout << "total time taken by the script to do solution calcuation for Air: "
            << duration_cast<ns>(t2b_air - t1b_air).count() << " ns" << std::endl;
  std::cout << "total time taken by the script to do solution calcuation for Atm: "
            << duration_cast<us>(t2b_atm - t1b_atm).count() / 1000 << " ms" << std::endl;
  std::cout << " " << std::endl;
  std::cout << "total time taken by the script to store rays: 0 ms" << std::endl;
  return 0;
}
