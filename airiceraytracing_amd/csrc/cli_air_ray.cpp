// AirRayTracing -- drop-in for the reference CLI (AirRayTracing.C): a Tx and an Rx both in the air.
// The launch-angle search is the Air2IceRayTracing one with the Rx height as the stop height and no
// ice leg (MinforLAng_params antennadepth = 0, AirRayTracing.C:53), so it runs as
// airice_rtf_eval(AIRICE_RTF_AIR2ICE, {TxHeight, distance, RxHeight, 0}) on the GPU; Tx below Rx
// swaps the two and reports 180 - angles (AirRayTracing.C:38-45, 147-157).
//
//   AirRayTracing <TxHeight m> <RxHeight m> <horizontal distance m>
//
// Reads Atmosphere.dat from the working directory, falling back to $AIRICE_ATMOSPHERE.
// PlotRayPath is false in the reference, so no path file is written.
#include <chrono>
#include <cstdlib>
#include <iostream>

#include "airice.h"

int main(int argc, char** argv) {
  const char* ex =
      "Here 5000 m is Tx Height in air in m, 3100 m is Rx Height in air, 1000 m is the horizontal "
      "distance btw Tx in air and Rx in air in m";
  if (argc == 1) {
    std::cout << "No Extra Command Line Argument Passed Other Than Program Name" << std::endl;
    std::cout << "Example run command: ./AirRayTracing 5000 3100 1000" << std::endl;
    std::cout << ex << std::endl;
    return 0;
  }
  if (argc < 4) {
    std::cout << "More Arguments needed!" << std::endl;
    std::cout << "Example run command: ./AirRayTracing 5000 3100 1000 3000" << std::endl;  // sic
    std::cout << ex << std::endl;
    return 0;
  }
  if (argc > 4) {
    std::cout << "More Arguments than needed!" << std::endl;
    std::cout << "Example run command: ./AirRayTracing 5000 3100 1000" << std::endl;
    std::cout << ex << std::endl;
    return 0;
  }
  std::cout << "Tx Height in air is set at " << std::atof(argv[1]) << " m, Rx Height in air is set at "
            << std::atof(argv[2]) << " m, Horizontal distance btw Tx and Rx is set at "
            << std::atof(argv[3]) << " m" << std::endl;
  const auto t1b = std::chrono::high_resolution_clock::now();
  const auto t1b_atm = std::chrono::high_resolution_clock::now();
  airice_medium m;
  if (airice_atmosphere_load("Atmosphere.dat", AIRICE_VARIANT_MULTIRAY, &m) != AIRICE_OK) {
    const char* env = std::getenv("AIRICE_ATMOSPHERE");
    if (env == nullptr || airice_atmosphere_load(env, AIRICE_VARIANT_MULTIRAY, &m) != AIRICE_OK) {
      std::cerr << "AirRayTracing: cannot read Atmosphere.dat: " << airice_last_error() << std::endl;
      return 1;
    }
  }
  const auto t2b_atm = std::chrono::high_resolution_clock::now();
  double AirTxHeight = std::atof(argv[1]);
  double AirRxHeight = std::atof(argv[2]);
  const double HorizontalDistance = std::atof(argv[3]);
  bool Flip = false;
  if (AirTxHeight < AirRxHeight) {
    const double SwitchHeight = AirTxHeight;
    AirTxHeight = AirRxHeight;
    AirRxHeight = SwitchHeight;
    Flip = true;
  }
  std::cout << AirTxHeight << " " << AirRxHeight << std::endl;
  const auto t1b_air = std::chrono::high_resolution_clock::now();
  const double args[4] = {AirTxHeight, HorizontalDistance, AirRxHeight, 0.0};
  double r[AIRICE_RTF_AIR2ICE_FIELDS];
  if (airice_rtf_eval(&m, AIRICE_RTF_AIR2ICE, args, 4, r, AIRICE_RTF_AIR2ICE_FIELDS) !=
      AIRICE_OK) {
    std::cerr << "AirRayTracing: " << airice_last_error() << std::endl;
    return 1;
  }
  const auto t2b_air = std::chrono::high_resolution_clock::now();
  std::cout << "startangle " << r[0] << " endangle " << r[1] << std::endl;
  std::cout << "Result from the minimization: Air Launch Angle: " << r[2] << " deg" << std::endl;
  const double IncidentAngleonRx = Flip ? 180 - r[4] : r[4];
  std::cout << " " << std::endl;
  std::cout << "***********Results for Air************" << std::endl;
  std::cout << "TotalHorizontalDistanceinAir " << r[3] << " m" << std::endl;
  std::cout << "IncidentAngleonRx " << IncidentAngleonRx << " deg" << std::endl;
  std::cout << "LvalueAir " << r[5] << std::endl;
  std::cout << "PropagationTimeAir " << r[6] << " ns" << std::endl;
  std::cout << " " << std::endl;
  using std::chrono::duration_cast;
  const auto t2b = std::chrono::high_resolution_clock::now();
  std::cout << "total time taken by the script to do solution calcuation: "
            << duration_cast<std::chrono::microseconds>(t2b - t1b).count() / 1000 << " ms"
            << std::endl;
  std::cout << "total time taken by the script to do solution calcuation for Air: "
            << duration_cast<std::chrono::nanoseconds>(t2b_air - t1b_air).count() << " ns"
            << std::endl;
  std::cout << "total time taken by the script to do solution calcuation for Atm: "
            << duration_cast<std::chrono::microseconds>(t2b_atm - t1b_atm).count() / 1000 << " ms"
            << std::endl;
  std::cout << " " << std::endl;
  std::cout << "total time taken by the script to store rays: 0 ms" << std::endl;
  return 0;
}
