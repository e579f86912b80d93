/*
 * AirIceRayTracing.h -- C++ drop-in for the reference's pythonwrapper library
 * (pythonwrapper/AirIceRayTracing.h:23-146, AirIceRayTracing.cc, TraceIceToAir.C), served by
 * libairice.so.  The reference builds libAirIceRayTracing.so from TraceIceToAir.C (which
 * #includes AirIceRayTracing.cc); its exported symbols are the AirIceRayTracing:: functions below,
 * the C++ TraceIceToAir and the extern "C" Py_TraceIceToAir (include/airice.h).  This header keeps
 * their names and signatures, hence the same Itanium-mangled names
 * (_ZN16AirIceRayTracing17Air2IceRayTracingEdddddPd,
 *  _ZN16AirIceRayTracing21GetRayTracingSolutionEddddRdS0_S0_S0_S0_S0_S0_S0_, _Z13TraceIceToAirddddPd, ...).
 *
 * Numerics: the pythonwrapper variant (AIRICE_VARIANT_PYWRAPPER): pi = 4*atan(1) (.h:25), metres
 * and degrees throughout, Air2IceRayTracing's own 15-slot output layout (.cc:1070-1084).
 *
 * Where each function runs:
 *   - One query per call, on the calling CPU thread by default: Air2IceRayTracing (.cc:929),
 *     GetRayTracingSolution (.cc:884), TraceIceToAir (TraceIceToAir.C:5) and the ray layer (fDnfR,
 *     ftimeD, fpathD, GetRay{Horizontal,Geometric}Path, GetRayPropagationTime,
 *     GetLayerHitPointPar, Get{Air,Ice}PropagationPar, MinimizeforLaunchAngle), from the same
 *     __host__ __device__ source as the GPU kernels (host sqrt and quotients: within about an ulp
 *     of a GPU batch's result).  AIRICE_SCALAR=device (airice_scalar_mode) runs each on a one-wave
 *     GPU kernel through the pinned scalar slot instead, bit-identical to the batch.  Batches run
 *     on the GPU: airice_solve_launch(AIRICE_VARIANT_PYWRAPPER), airice_trace_ice_to_air_launch.
 *   - Host: the atmosphere readers, n(z) and the layer scans, Fresnel coefficients, and
 *     FindFunctionRoot (GSL bisection / Brent on the caller's host function, airice_gsl_roots.h).
 *
 * Namespace data.  The reference defines it as header statics (.h:29-72: one copy per translation
 * unit, so a caller's writes never reached the library's copy).  Here it is one shared copy,
 * filled by MakeAtmosphere(file), and read by every call: a caller that changes B_air, C_air,
 * ATMLAY, MaxLayers, A_air, A_const or UseConstantRefractiveIndex after MakeAtmosphere changes the
 * medium of the following calls (e.g. the constant-index set-up commented out at
 * TraceIceToAir.C:27-29).  A caller that never writes them gets exactly the reference library's
 * behaviour.  With UseConstantRefractiveIndex set, A_const must equal A_air (as in that set-up).
 *
 * Logging: the reference prints one block per TraceIceToAir call (TraceIceToAir.C:35-55); this
 * library is quiet unless AIRICE_VERBOSE=1.
 */
#ifndef AIRICE_AIRICERAYTRACING_H
#define AIRICE_AIRICERAYTRACING_H

#include <cmath>
#include <string>
#include <vector>

#include "airice_gsl_roots.h"

namespace AirIceRayTracing {

static const double pi = 4.0 * atan(1.0); /* .h:25 */
static const double spedc = 299792458.0;  /* .h:26 */

/* refractive-index profile of the atmosphere file (.h:29-31), filled by readnhFromFile() */
extern std::vector<std::vector<double>> nh_data;
extern std::vector<std::vector<double>> lognh_data;
extern std::vector<std::vector<double>> h_data;
/* ATMLAY (cm) and the mass-overburden a,b,c rows (.h:34-35), the fitted air model (.h:38-39) */
extern double ATMLAY[5];
extern double abc[5][3];
extern double C_air[5];
extern double B_air[5];
extern int MaxLayers; /* .h:46 */

/* Both read the named GDAS file (.cc:4-128). */
int readATMpar(std::string atmosFileName);
int readnhFromFile(std::string atmosFileName);

extern bool UseConstantRefractiveIndex; /* .h:54 */
static const double A_ice = 1.78;       /* .h:57 */
double GetB_ice(double z);
double GetC_ice(double z);
double Getnz_ice(double z);

extern double A_air;   /* .h:69 */
extern double A_const; /* .h:72 */

/* N0 = the natural cubic spline of the last MakeAtmosphere()'s profile at 0 m, then B_air chained
 * for continuity with the current A_air (.cc:154-170). */
int FillInAirRefractiveIndex();
double GetB_air(double z);
double GetC_air(double z);
double Getnz_air(double z);

/* Fresnel amplitude coefficients (.cc:242-312), thetai in radians. */
double Refl_S(double thetai, double IceLayerHeight);
double Trans_S(double thetai, double IceLayerHeight);
double Refl_P(double thetai, double IceLayerHeight);
double Trans_P(double thetai, double IceLayerHeight);

/* GSL root-solver driver (.cc:315-353): set, then {iterate; root; x_lower; x_upper;
 * gsl_root_test_interval(lo, hi, 0, tolerance)} while CONTINUE and iter < iterations. */
double FindFunctionRoot(gsl_function F, double x_lo, double x_hi, const gsl_root_fsolver_type* T,
                        double tolerance, int iterations);

struct fDnfR_params { double a, b, c, l; };
double fDnfR(double x, void* params);
struct ftimeD_params { double a, b, c, speedc, l; int airorice; };
double ftimeD(double x, void* params);
double fpathD(double x, void* params);

double GetRayHorizontalPath(double A, double RxDepth, double TxDepth, double Lvalue, int AirOrIce);
double GetRayPropagationTime(double A, double RxDepth, double TxDepth, double Lvalue, int AirOrIce);
double GetRayGeometricPath(double A, double RxDepth, double TxDepth, double Lvalue, int AirOrIce);

/* new double[5] {THD, receive angle deg, L, time s, geometric path}; the caller delete[]s it */
double* GetLayerHitPointPar(double n_layer1, double RxDepth, double TxDepth, double IncidentAng,
                            int AirOrIce);

std::vector<double> flatten(const std::vector<std::vector<double>>& v);

/* Reads the named GDAS file (readATMpar, readnhFromFile, spline, FillInAirRefractiveIndex). */
int MakeAtmosphere(std::string atmosFileName);

/* new double[5*MaxLayers+2] (per layer the five of GetLayerHitPointPar, filled-layer count at
 * [5*MaxLayers+1]) / new double[5]; the caller delete[]s them */
double* GetAirPropagationPar(double LaunchAngle, double AirTxHeight, double IceLayerHeight);
double* GetIcePropagationPar(double IncidentAngleonIce, double IceLayerHeight, double AntennaDepth,
                             double Lvalue);

struct MinforLAng_params { double airtxheight, icelayerheight, antennadepth, horizontaldistance; };
double MinimizeforLaunchAngle(double x, void* params);

/* m / degrees (.cc:884-927): the launch-angle solve with thR formed as the reference does, then
 * the eight outputs and CheckSolution. */
bool GetRayTracingSolution(double SrcHeightASL, double HorizontalDistanceToRx,
                           double RxDepthBelowIceBoundary, double IceLayerHeight,
                           double& opticalPathLengthInIce, double& opticalPathLengthInAir,
                           double& geometricalPathLengthInIce, double& geometricalPathLengthInAir,
                           double& launchAngle, double& horizontalDistanceToIntersectionPoint,
                           double& AngleOfIncidenceOnIce, double& RecievedAngleInIce);

/* .cc:929-1086: fills dummy[0..14]. */
void Air2IceRayTracing(double AirTxHeight, double HorizontalDistance, double IceLayerHeight,
                       double AntennaDepth, double StraightAngle, double dummy[20]);

}  // namespace AirIceRayTracing

/* TraceIceToAir.C:5-73: MakeAtmosphere("Atmosphere.dat") (fallback $AIRICE_ATMOSPHERE; the parsed
 * file is cached while its size and mtime are unchanged), GetRayTracingSolution, the
 * launch/receive swap, ArrayParameters[10] (-1000 everywhere when there is no solution). */
void TraceIceToAir(double AntennaDepth, double IceLayerHeight, double AirTxHeight,
                   double HorizontalDistance, double ArrayParameters[10]);

#endif /* AIRICE_AIRICERAYTRACING_H */
