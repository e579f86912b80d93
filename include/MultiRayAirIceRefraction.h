/*
 * MultiRayAirIceRefraction.h -- C++ drop-in surface of libairice.so for CoREAS-style callers.
 *
 * Same namespace, function names, signatures, units and globals as the reference's
 * MultiRayAirIceRefraction.h/.cc (uzairlatif90/AirIceRayTracing), so existing call sites
 * (e.g. RunMultiRayCode.C:29-59) compile and link against libairice.so unchanged, minus the
 * `#include "MultiRayAirIceRefraction.cc"` line.  The hot path -- MakeRayTracingTable
 * (.cc:2019), GetRayTracingSolutions (.cc:1796), Air2IceRayTracing (.cc:1464),
 * GetHorizontalDistanceToIntersectionPoint (.cc:945) and its table variant _Table (.cc:1305)
 * -- runs on the MI355X.
 *
 * Not provided: the GSL-typed internals (FindFunctionRoot, gsl_* statics) and the helpers
 * that return heap scratch arrays (GetLayerHitPointPar, Get{Air,Ice}PropagationPar,
 * fDnfR/ftimeD/fpathD, MinimizeforLaunchAngle); they are implementation details of the
 * reference's CPU solver with no caller outside it.  The deprecated MakeTable /
 * GetInterpolatedValue (.cc:1618-1794, "Do not use this function") are not provided.
 *
 * Units (as the reference): CoREAS-facing functions take and return cm and radians;
 * Air2IceRayTracing / GetRayTracingSolutions take m and degrees.  AntennaDepth < 0 means
 * the receiver is below the ice surface.
 */
#ifndef AIRICE_MULTIRAYAIRICEREFRACTION_H
#define AIRICE_MULTIRAYAIRICEREFRACTION_H

#include <cstddef>
#include <vector>

/* Defined by the caller (reference .h:23-24, RunMultiRayCode.C:3-4). */
extern std::vector<double> AntennaDepths;
extern std::vector<int> AntennaTableAlreadyMade;

/* Library globals (reference .cc:3-21). */
extern double MaxAirTxHeight;
extern double MinAirTxHeight;
extern std::vector<std::vector<std::vector<float>>> AllTableAllAntData;
extern double AngleStepSize;
extern double LoopStartAngle;
extern double LoopStopAngle;
extern int TotalAngleSteps;
extern double HeightStepSize;
extern double LoopStartHeight;
extern double LoopStopHeight;
extern int TotalHeightSteps;

namespace MultiRayAirIceRefraction {

static const double pi = 3.1415927;       /* .h:29 (sic: not M_PI) */
static const double spedc = 299792458.0;  /* .h:30 */
static const double A_ice_def = 1.78;
static const double B_ice_def = -0.43;
static const double C_ice_def = 0.0132;
static constexpr double TransitionBoundary = 0;
static const double A_air = 1.00;

/* Reads "Atmosphere.dat" from the working directory (falls back to $AIRICE_ATMOSPHERE). */
int MakeAtmosphere();

double GetB_ice(double z);
double GetC_ice(double z);
double Getnz_ice(double z);
double GetB_air(double z);
double GetC_air(double z);
double Getnz_air(double z);

/* Fresnel amplitude coefficients (.cc:267-337), thetai in radians. */
double Refl_S(double thetai, double IceLayerHeight);
double Trans_S(double thetai, double IceLayerHeight);
double Refl_P(double thetai, double IceLayerHeight);
double Trans_P(double thetai, double IceLayerHeight);

/* CoREAS entry (cm in, cm/rad out), solved on the GPU. */
bool GetHorizontalDistanceToIntersectionPoint(
    double SrcHeightASL, double HorizontalDistanceToRx, double RxDepthBelowIceBoundary,
    double IceLayerHeight, double& opticalPathLengthInIce, double& opticalPathLengthInAir,
    double& geometricalPathLengthInIce, double& geometricalPathLengthInAir, double& launchAngle,
    double& horizontalDistanceToIntersectionPoint, double& transmissionCoefficientS,
    double& transmissionCoefficientP, double& RecievedAngleInIce);

double oneDLinearInterpolation(double x, double xa, double ya, double xb, double yb);

/* Air2IceRayTracing (.cc:1464): m / degrees; fills dummy[0..16]. */
void Air2IceRayTracing(double AirTxHeight, double HorizontalDistance, double IceLayerHeight,
                       double AntennaDepth, double StraightAngle, double dummy[20]);

/* GetRayTracingSolutions (.cc:1796): one forward ray; fills dummy[0..17]. */
void GetRayTracingSolutions(double RayLaunchAngleInAir, double AirTxHeight, double IceLayerHeight,
                            double AntennaDepth, double dummy[20], bool& InIce);

/* MakeRayTracingTable (.cc:2019): cm in; appends the 11-column float table of this antenna to
 * AllTableAllAntData using the grid globals above (the reference's defaults: 100 km to the ice
 * in 10 m steps x 90.1..180 deg in 0.1 deg steps).  Returns 0. */
int MakeRayTracingTable(double AntennaDepth, double IceLayerHeight, int AntennaNumber);

/* Table lookup on an already-resolved table index (AllTableAllAntData[TableIndex]), run on the
 * GPU against the table's HBM copy (kept from MakeRayTracingTable, or uploaded on first use
 * when AllTableAllAntData[TableIndex] was filled by the caller).  Same outputs, units, globals
 * (MaxAirTxHeight / MinAirTxHeight are set) and quirks as the reference (.cc:1305-1462). */
bool TableLookup(double SrcHeightASL, double HorizontalDistanceToRx,
                 double RxDepthBelowIceBoundary, double IceLayerHeight, int TableIndex,
                 double& opticalPathLengthInIce, double& opticalPathLengthInAir,
                 double& geometricalPathLengthInIce, double& geometricalPathLengthInAir,
                 double& launchAngle, double& horizontalDistanceToIntersectionPoint,
                 double& transmissionCoefficientS, double& transmissionCoefficientP,
                 double& RecievedAngleInIce);

/* Batched form: n queries (cm) against one resolved table; out is n rows of the 9 outputs in
 * the reference's argument order; ok[i] the returned bool.  One launch for the whole batch. */
void TableLookupBatch(const double* SrcHeightASL, const double* HorizontalDistanceToRx,
                      const double* RxDepthBelowIceBoundary, double IceLayerHeight, int TableIndex,
                      size_t n, double* out9, bool* ok);

/* GetHorizontalDistanceToIntersectionPoint_Table (.cc:1305).  The antenna -> table remap reads
 * the caller-owned AntennaDepths / AntennaTableAlreadyMade (.cc:1348-1352), so it is compiled
 * into the caller here; the lookup itself runs in libairice.so. */
inline bool GetHorizontalDistanceToIntersectionPoint_Table(
    double SrcHeightASL, double HorizontalDistanceToRx, double RxDepthBelowIceBoundary,
    double IceLayerHeight, int AntennaNumber, double& opticalPathLengthInIce,
    double& opticalPathLengthInAir, double& geometricalPathLengthInIce,
    double& geometricalPathLengthInAir, double& launchAngle,
    double& horizontalDistanceToIntersectionPoint, double& transmissionCoefficientS,
    double& transmissionCoefficientP, double& RecievedAngleInIce) {
  for (int j = 0; j < (int)AntennaTableAlreadyMade.size(); j++) {
    if (AntennaDepths[AntennaNumber] == AntennaDepths[AntennaTableAlreadyMade[j]]) {
      AntennaNumber = j;
    }
  }
  return TableLookup(SrcHeightASL, HorizontalDistanceToRx, RxDepthBelowIceBoundary,
                     IceLayerHeight, AntennaNumber, opticalPathLengthInIce,
                     opticalPathLengthInAir, geometricalPathLengthInIce,
                     geometricalPathLengthInAir, launchAngle,
                     horizontalDistanceToIntersectionPoint, transmissionCoefficientS,
                     transmissionCoefficientP, RecievedAngleInIce);
}

}  // namespace MultiRayAirIceRefraction

#endif
