/* RayTracingFunctions.h -- drop-in for the reference's RayTracingFunctions:: namespace
 * (RayTracingFunctions.h / RayTracingFunctions.cc, the library behind the cfg1
 * SingleRayAirIceRefraction CLI), served by libairice.so.
 *
 * Same names, signatures, units and output layouts as the reference:
 *   - GetLayerHitPointPar / GetIcePropagationPar return new double[4] {THD, receive angle (deg),
 *     L, time (s)}; GetAirPropagationPar returns new double[4*MaxLayers+1] with the filled-layer
 *     count at [4*MaxLayers].  The caller delete[]s them, as with the reference.
 *   - Every ray quantity (fDnfR, ftimeD, GetRayOpticalPath, GetRayPropagationTime, the three
 *     *Par functions, MinimizeforLaunchAngle) is one query per call with the reference's
 *     expressions (airice_rtf_eval, include/airice.h), on the calling CPU thread by default; with
 *     AIRICE_SCALAR=device (or airice_scalar_mode(AIRICE_SCALAR_DEVICE)) on a one-wave GPU
 *     kernel per call.  The host form is the same __host__ __device__ source with the host's
 *     correctly rounded sqrt and quotients: within about an ulp of the GPU's.  Batches run on the
 *     GPU through the batched C-ABI (airice_single_ray_*, airice_solve_*, airice_table_*).
 *   - MakeAtmosphere() reads "Atmosphere.dat" from the working directory (fallback
 *     $AIRICE_ATMOSPHERE) and fills ATMLAY, abc, B_air, C_air, MaxLayers, h_data, nh_data,
 *     lognh_data.  The reference defines these as header statics; here they are one shared copy.
 * FindFunctionRoot (.cc:256-290, max_iter 20) keeps its GSL-typed signature (airice_gsl_roots.h)
 * and runs GSL's bisection / Brent on the caller's host function.  Not provided: the GSL
 * spline/accelerator statics (GSL objects; N0 comes from the library's own spline).
 * Link: -L<repo>/airiceraytracing_amd -lairice. */
#ifndef AIRICE_RAYTRACINGFUNCTIONS_H_
#define AIRICE_RAYTRACINGFUNCTIONS_H_

#include <vector>

#include "airice_gsl_roots.h"

namespace RayTracingFunctions {

static constexpr double pi = 3.1415927;    /* RayTracingFunctions.h:25 */
static constexpr double spedc = 299792458.0; /* .h:26 */
static constexpr double A_ice = 1.78;      /* .h:56 */
static constexpr double A_air = 1.00;      /* .h:68 */

/* atmosphere data (.h:29-45) */
extern std::vector<std::vector<double>> nh_data;
extern std::vector<std::vector<double>> lognh_data;
extern std::vector<std::vector<double>> h_data;
extern double ATMLAY[5];
extern double abc[5][3];
extern double C_air[5];
extern double B_air[5];
extern int MaxLayers;

int readATMpar();
int readnhFromFile();
double GetB_ice(double z);
double GetC_ice(double z);
double Getnz_ice(double z);
int FillInAirRefractiveIndex();
double GetB_air(double z);
double GetC_air(double z);
double Getnz_air(double z);
double Refl_S(double thetai, double IceLayerHeight);
double Refl_P(double thetai, double IceLayerHeight);

double FindFunctionRoot(gsl_function F, double x_lo, double x_hi, const gsl_root_fsolver_type *T,
                        double tolerance);

struct fDnfR_params { double a, b, c, l; };
double fDnfR(double x, void *params);
struct ftimeD_params { double a, b, c, speedc, l; int airorice; };
double ftimeD(double x, void *params);

double GetRayOpticalPath(double A, double RxDepth, double TxDepth, double Lvalue, int AirOrIce);
double GetRayPropagationTime(double A, double RxDepth, double TxDepth, double Lvalue, int AirOrIce);
double *GetLayerHitPointPar(double n_layer1, double RxDepth, double TxDepth, double IncidentAng,
                            int AirOrIce);

std::vector<double> flatten(const std::vector<std::vector<double>> &v);
int MakeAtmosphere();
double *GetAirPropagationPar(double LaunchAngle, double AirTxHeight, double IceLayerHeight);
double *GetIcePropagationPar(double IncidentAngleonIce, double IceLayerHeight, double AntennaDepth,
                             double Lvalue);

struct MinforLAng_params { double airtxheight, icelayerheight, antennadepth, horizontaldistance; };
double MinimizeforLaunchAngle(double x, void *params);

}  // namespace RayTracingFunctions

#endif /* AIRICE_RAYTRACINGFUNCTIONS_H_ */
