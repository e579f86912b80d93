/*
 * MultiRayAirIceRefraction.h -- C++ drop-in surface of libairice.so for CoREAS-style callers.
 *
 * Same namespace, function names, signatures (hence mangled names), units and globals as the
 * reference's MultiRayAirIceRefraction.h/.cc (uzairlatif90/AirIceRayTracing), so existing call
 * sites (e.g. RunMultiRayCode.C:29-59) compile and link against libairice.so unchanged, minus the
 * `#include "MultiRayAirIceRefraction.cc"` line.
 *
 * Where each function runs:
 *   - GPU, always: MakeRayTracingTable (.cc:2019) and the extensions MakeRayTracingTables and
 *     TableLookupBatch below -- the batch entry points (one launch chain per call).
 *   - The calling CPU thread, by default (airice_scalar_mode, include/airice.h): every one-query
 *     call -- GetRayTracingSolutions (.cc:1796), Air2IceRayTracing (.cc:1464),
 *     GetHorizontalDistanceToIntersectionPoint (.cc:945) and the ray layer (fDnfR, ftimeD,
 *     fpathD, GetRay{Horizontal,Geometric}Path, GetRayPropagationTime, GetLayerHitPointPar,
 *     Get{Air,Ice}PropagationPar, MinimizeforLaunchAngle).  They are compiled from the same
 *     __host__ __device__ source as the GPU kernels, with the host's correctly rounded sqrt and
 *     quotients, so a result can differ from the same query inside a GPU batch by about an ulp
 *     (within the 1e-9 contract; the launch angle is the same GSL bisection's).
 *     AIRICE_SCALAR=device in the environment, or airice_scalar_mode(AIRICE_SCALAR_DEVICE), sends
 *     them to one-wave GPU kernels instead (bit-identical to the batch, ~10-20 us per call).
 *   - Host, from the same source the batch lookup kernel is compiled from (airice_lookup.hpp):
 *     GetHorizontalDistanceToIntersectionPoint_Table (.cc:1305), GetParValues (.cc:1172),
 *     FindClosestAirTxHeight (.cc:1033), FindClosestTHD (.cc:1128) -- table walks over the
 *     caller's host AllTableAllAntData, bit-identical to the device lookup; a query that reaches
 *     the reference's minimizer fallback (.cc:1418) runs that solve where the mode above says.
 *     Extrapolate / FindExtrapolationLimit (.cc:997-1031) and the atmosphere file readers are host
 *     code as in the reference.
 *
 * FindFunctionRoot (.cc:340-374) keeps its GSL-typed signature (airice_gsl_roots.h) and runs GSL's
 * bisection / Brent on the caller's host function.  Not provided: the gsl_interp_accel /
 * gsl_spline statics (GSL objects; N0 comes from the library's own spline), and the deprecated
 * MakeTable / GetInterpolatedValue (.cc:1618-1794, "Do not use this function").
 *
 * Namespace data: the reference defines it as header statics (one copy per translation unit,
 * .h:33-81); here it is one shared copy, filled by MakeAtmosphere().  A_ice / B_ice / C_ice are
 * read by every call, so a caller that changes them (as the reference allows) changes the ice
 * model of the following calls and tables.
 *
 * Units (as the reference): CoREAS-facing functions take and return cm and radians;
 * Air2IceRayTracing / GetRayTracingSolutions take m and degrees.  AntennaDepth < 0 means
 * the receiver is below the ice surface.
 */
#ifndef AIRICE_MULTIRAYAIRICEREFRACTION_H
#define AIRICE_MULTIRAYAIRICEREFRACTION_H

#include <cstddef>
#include <vector>

#include "airice_gsl_roots.h"

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

/* refractive-index profile of Atmosphere.dat (.h:33-35), filled by readnhFromFile() */
extern std::vector<std::vector<double>> nh_data;
extern std::vector<std::vector<double>> lognh_data;
extern std::vector<std::vector<double>> h_data;
/* interpolation grid of the deprecated MakeTable (.h:38-53), kept with the reference's values */
extern std::vector<double> GridPositionH;
extern std::vector<double> GridPositionTh;
extern std::vector<double> GridZValue[10];
extern double GridStartTh, GridStopTh, GridStepSizeH_O, GridStepSizeTh_O, GridWidthH, GridWidthTh;
extern int GridPoints, TotalStepsH_O, TotalStepsTh_O;
extern double GridStartH, GridStopH;
/* ATMLAY and the mass-overburden a,b,c rows (.h:56-57), the fitted air model (.h:60-61) */
extern double ATMLAY[5];
extern double abc[5][3];
extern double C_air[5];
extern double B_air[5];
static const double A_ice_def = 1.78;
static const double B_ice_def = -0.43;
static const double C_ice_def = 0.0132;
static constexpr double TransitionBoundary = 0;
extern double A_ice; /* .h:75-77: A_ice_def, B_ice_def, C_ice_def */
extern double B_ice;
extern double C_ice;
extern int MaxLayers; /* .h:84 */
static const double A_air = 1.00;

int readATMpar();
int readnhFromFile();
int FillInAirRefractiveIndex();
std::vector<double> flatten(const std::vector<std::vector<double>>& v);

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

/* CoREAS entry (cm in, cm/rad out): one query, on the calling thread (see above). */
bool GetHorizontalDistanceToIntersectionPoint(
    double SrcHeightASL, double HorizontalDistanceToRx, double RxDepthBelowIceBoundary,
    double IceLayerHeight, double& opticalPathLengthInIce, double& opticalPathLengthInAir,
    double& geometricalPathLengthInIce, double& geometricalPathLengthInAir, double& launchAngle,
    double& horizontalDistanceToIntersectionPoint, double& transmissionCoefficientS,
    double& transmissionCoefficientP, double& RecievedAngleInIce);

double oneDLinearInterpolation(double x, double xa, double ya, double xb, double yb);

/* GSL root-solver driver (.cc:340-374, max_iter 40): bisection or Brent, by the solver's name. */
double FindFunctionRoot(gsl_function F, double x_lo, double x_hi, const gsl_root_fsolver_type* T,
                        double tolerance);

/* The ray layer (.cc:377-917), one query per call (see above).  *Par functions return new[]'d arrays the
 * caller delete[]s, as with the reference: GetLayerHitPointPar / GetIcePropagationPar 5 doubles
 * {THD, receive angle deg, L, time s, geometric path}; GetAirPropagationPar 5 x MaxLayers + 2,
 * per layer the same five, the filled-layer count at [5 * MaxLayers + 1]. */
struct fDnfR_params { double a, b, c, l; };
double fDnfR(double x, void* params);
struct ftimeD_params { double a, b, c, speedc, l; int airorice; };
double ftimeD(double x, void* params);
double fpathD(double x, void* params);
double GetRayHorizontalPath(double A, double RxDepth, double TxDepth, double Lvalue, int AirOrIce);
double GetRayPropagationTime(double A, double RxDepth, double TxDepth, double Lvalue, int AirOrIce);
double GetRayGeometricPath(double A, double RxDepth, double TxDepth, double Lvalue, int AirOrIce);
double* GetLayerHitPointPar(double n_layer1, double RxDepth, double TxDepth, double IncidentAng,
                            int AirOrIce);
double* GetAirPropagationPar(double LaunchAngle, double AirTxHeight, double IceLayerHeight);
double* GetIcePropagationPar(double IncidentAngleonIce, double IceLayerHeight, double AntennaDepth,
                             double Lvalue);
struct MinforLAng_params { double airtxheight, icelayerheight, antennadepth, horizontaldistance; };
double MinimizeforLaunchAngle(double x, void* params);

/* Table walks (.cc:997-1302) over AllTableAllAntData[AntennaNumber] and the grid globals of the
 * last table made; run on the host with the batch lookup kernel's own code. */
double Extrapolate(int Par, int index, double TotalHorizontalDistance, int AntennaNumber);
double FindExtrapolationLimit(int index, double TotalHorizontalDistance, int AntennaNumber);
void FindClosestAirTxHeight(double ParValue, int& RStartIndex1, int& REndIndex1,
                            double& ClosestVal1, int& RStartIndex2, int& REndIndex2,
                            double& ClosestVal2, int AntennaNumber);
int FindClosestTHD(double ParValue, int StartIndex, int EndIndex, int& RStartIndex,
                   int& REndIndex, double& ClosestVal, int AntennaNumber);
int GetParValues(double AntennaNumber, double AirTxHeight, double TotalHorizontalDistance,
                 double IceLayerHeight, double& AirTxHeight1, double Par1[10],
                 double& AirTxHeight2, double Par2[10]);

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

/* GetHorizontalDistanceToIntersectionPoint_Table (.cc:1305-1462): the antenna -> table remap
 * over the caller's AntennaDepths / AntennaTableAlreadyMade (.cc:1348-1352), then one lookup on
 * the host (see above).  Same outputs, units, globals (MaxAirTxHeight / MinAirTxHeight) and
 * quirks as the reference. */
bool GetHorizontalDistanceToIntersectionPoint_Table(
    double SrcHeightASL, double HorizontalDistanceToRx, double RxDepthBelowIceBoundary,
    double IceLayerHeight, int AntennaNumber, double& opticalPathLengthInIce,
    double& opticalPathLengthInAir, double& geometricalPathLengthInIce,
    double& geometricalPathLengthInAir, double& launchAngle,
    double& horizontalDistanceToIntersectionPoint, double& transmissionCoefficientS,
    double& transmissionCoefficientP, double& RecievedAngleInIce);

/* Extensions (no reference counterpart). */
/* MakeRayTracingTable for several antennas in ONE GPU launch (airice_table_launch_multi): appends
 * one table per entry of AntennaDepth (cm, in order) to AllTableAllAntData, exactly as the
 * reference's per-antenna loop of MakeRayTracingTable calls would (RunMultiRayCode.C:29-52), with
 * one launch ramp and drain for all of them.  The grid globals are those of the last antenna. */
int MakeRayTracingTables(const std::vector<double>& AntennaDepth, double IceLayerHeight);
/* The same lookup on an already-resolved table index (AllTableAllAntData[TableIndex]). */
bool TableLookup(double SrcHeightASL, double HorizontalDistanceToRx,
                 double RxDepthBelowIceBoundary, double IceLayerHeight, int TableIndex,
                 double& opticalPathLengthInIce, double& opticalPathLengthInAir,
                 double& geometricalPathLengthInIce, double& geometricalPathLengthInAir,
                 double& launchAngle, double& horizontalDistanceToIntersectionPoint,
                 double& transmissionCoefficientS, double& transmissionCoefficientP,
                 double& RecievedAngleInIce);

/* Batched form on the GPU: n queries (cm) against one resolved table; out is n rows of the 9
 * outputs in the reference's argument order; ok[i] the returned bool.  One launch chain for the
 * whole batch against the table's HBM copy (kept from MakeRayTracingTable; a table the caller
 * filled or changed is uploaded again). */
void TableLookupBatch(const double* SrcHeightASL, const double* HorizontalDistanceToRx,
                      const double* RxDepthBelowIceBoundary, double IceLayerHeight, int TableIndex,
                      size_t n, double* out9, bool* ok);

}  // namespace MultiRayAirIceRefraction

#endif
