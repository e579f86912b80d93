/*
 * airice_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement ("oracle") of the uzairlatif90/AirIceRayTracing hot path:
 * MultiRayAirIceRefraction table rays + Air2Ice launch-angle bisection, and the
 * pythonwrapper (AirIceRayTracing::) variant.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the checker /
 * CPU baseline.  The product path (airiceraytracing_amd/, libairice.so) never
 * links or calls it.
 *
 * Parity status: the reference needs GNU GSL (absent from this image), so it is
 * unbuildable here; the oracle is a restatement pinned by (a) scipy's natural
 * cubic spline for the atmosphere N0, (b) the known-answer values recorded in
 * SURVEY.md §4 (see tests/golden/README.md for their provenance), and (c) numerical
 * integration of the ray equations in its own n(z) (tests/test_oracle_physics.py:
 * segment closed forms, whole forward rays, Air2Ice roots).
 *
 * Every function cites the reference file:line it restates.  Faithful mode: the
 * call structure mirrors the reference (per-call layer scans, repeated libm calls),
 * so its timing stands in for the reference CPU path.
 */
#ifndef AIRICE_ORACLE_H
#define AIRICE_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Atmosphere + ice medium (MultiRayAirIceRefraction.h:57-81, .cc:24-213). */
typedef struct or_medium {
  double atmlay[5];    /* ATMLAY, cm (ATMLAY[4] forced to 1.5e7, .cc:66) */
  double abc[5][3];    /* mass-overburden a,b,c (abc[4]=abc[3], .cc:62-64) */
  double C_air[5];     /* .cc:198 */
  double B_air[5];     /* .cc:200-205 */
  double N0;           /* natural cubic spline n(h=0), .cc:203 */
  int    max_layers;   /* |h_data|+1, .cc:142 */
  int    n_points;     /* flattened spline knots */
  int    layer_sizes[8];
  double A_air;        /* .h:99 */
  double A_ice, B_ice, C_ice;  /* .h:64-66 */
  double pi;           /* 3.1415927 (MultiRay/RTF) or 4*atan(1) (pythonwrapper) */
  double h_top;        /* h_data.back().back(): last tabulated height, m
                          (SingleRayAirIceRefraction.C:40-45 clamps the Tx to it) */
  int    constant_air_index; /* pythonwrapper AirIceRayTracing::UseConstantRefractiveIndex
                                (.h:54): GetB_air = 0, GetC_air = 1e-9, Getnz_air = A_const,
                                bracket [90, thR] without the probe loop (.cc:178-239, 955-982) */
  double A_const;      /* pythonwrapper .h:72 */
} or_medium;

/* Status codes of one bisection solve (GSL 2.x bisection semantics). */
enum {
  OR_SOLVE_OK = 0,            /* bracket finite; loop ended on test_interval or max_iter */
  OR_SOLVE_NONFINITE_END = 1, /* f(lo) or f(hi) non-finite: reference reads uninitialised
                                 GSL state (UB) -> row unpinned; we model zeroed state */
  OR_SOLVE_BAD_BRACKET = 2,   /* lo > hi: gsl_root_fsolver_set fails (UB downstream) */
  OR_SOLVE_STALE_MID = 4,     /* a midpoint f was non-finite; root frozen (GSL EBADFUNC) */
  OR_SOLVE_PROBED = 8,        /* the 0.05-degree bracket-probe loop ran (.cc:1490-1511) */
  OR_SOLVE_MAXITER = 16,      /* 40 iterations without test_interval success */
  OR_SOLVE_NO_AIR_LAYER = 32  /* no air layer between Tx and ice (reference reads out[-4]) */
};

/* Parse a GDAS Atmosphere.dat text image (readATMpar .cc:24-71, readnhFromFile
 * .cc:73-147, flatten .cc:649, spline .cc:931-933, FillInAirRefractiveIndex .cc:193).
 * pi selects the variant constant.  Returns 0 on success. */
int or_parse_atmosphere(const char *text, size_t len, double pi, or_medium *m);
int or_load_atmosphere(const char *path, double pi, or_medium *m);

/* Natural cubic spline of the flattened profile evaluated at x (GSL cspline). */
double or_spline_eval_at(const double *xa, const double *ya, int n, double x);

/* Scalar pieces (exposed for unit tests). */
double or_getnz_air(const or_medium *m, double z);
double or_getnz_ice(const or_medium *m, double z);
void   or_layer_hit_point_par(const or_medium *m, double n_layer1, double rx, double tx,
                              double inc_deg, int air_or_ice, double out[5]);

/* GetRayTracingSolutions (.cc:1796-2017): dummy[18]. */
void or_ray_solution(const or_medium *m, double launch_deg, double txh, double ice_h,
                     double depth, int in_ice, double dummy[18]);

/* MakeRayTracingTable grid (.cc:12-21, 2019-2061). */
typedef struct or_grid {
  double start_height, stop_height, height_step;
  int    height_steps;
  double start_angle, stop_angle, angle_step;
  int    angle_steps;
  double depth_m, ice_m;
  int    in_ice;
  int    table_rows;   /* rows with Tx height > 0 (.cc:2082): the table is this prefix */
} or_grid;
void or_grid_init(or_grid *g, double depth_cm, double ice_cm, double height_step,
                  double start_angle, double stop_angle, double angle_step);
/* Rays [row0,row1) x all angles; table: 11 float columns (col stride = ld);
 * full (nullable): 18 double columns (col stride = ld). nthreads<=0 -> serial. */
void or_table_rows(const or_medium *m, const or_grid *g, int row0, int row1,
                   float *table, double *full, size_t ld, int nthreads);

/* Air2IceRayTracing (.cc:1464-1616): dummy[17], returns status bits. */
int or_air2ice(const or_medium *m, double txh, double dist, double ice_h, double depth,
               double straight_angle, double dummy[17]);
/* Generic GSL-bisection driver (FindFunctionRoot .cc:340-374), exposed for unit tests. */
typedef double (*or_fn)(double x, void *ctx);
/* GSL 2.x Brent under RayTracingFunctions::FindFunctionRoot; *iters = iterations run. */
double or_brent(or_fn f, void *ctx, double x_lo, double x_hi, double tol_rel, int max_iter,
                int *status, int *iters);
/* Air2IceRayTracing CLI solve (Air2IceRayTracing.C:56-185); out[16] as AIRICE_RTF_AIR2ICE. */
void or_rtf_air2ice(const or_medium *m, double AirTxHeight, double HorizontalDistance,
                    double IceLayerHeight, double AntennaDepth, double *out);
double or_bisect(or_fn f, void *ctx, double x_lo, double x_hi, double tol, int max_iter,
                 int *status);
/* thR of GetHorizontalDistanceToIntersectionPoint (.cc:952-958), metres. */
double or_straight_angle(const or_medium *m, double txh, double dist, double ice_h, double depth);
/* Batched minimizer over (txh, dist, depth) metres; out: 17 double columns (stride ld). */
void or_solve_batch(const or_medium *m, const double *txh, const double *dist,
                    const double *depth, double ice_h, size_t n, double *out, size_t ld,
                    uint8_t *status, int nthreads);

/* GetHorizontalDistanceToIntersectionPoint (.cc:945-989), cm in, outs[9], returns bool. */
int or_hdtip(const or_medium *m, double src_cm, double dist_cm, double depth_cm,
             double ice_cm, double outs[9]);
/* The same over a batch (OpenMP): out 9 columns (stride ld), ok[], status[] (solve status bits). */
void or_hdtip_batch(const or_medium *m, const double *src_cm, const double *dist_cm,
                    const double *depth_cm, double ice_cm, size_t n, double *out, size_t ld,
                    uint8_t *ok, uint8_t *status, int nthreads);

/* pythonwrapper variant: AirIceRayTracing::Air2IceRayTracing (AirIceRayTracing.cc:929-1086),
 * dummy[15]; TraceIceToAir (TraceIceToAir.C:5-73) -> ArrayParameters[10]. */
int or_py_air2ice(const or_medium *m, double txh, double dist, double ice_h, double depth,
                  double straight_angle, double dummy[15]);
int or_py_trace_ice_to_air(const or_medium *m, double depth, double ice_h, double txh,
                           double dist, double out10[10]);
void or_py_trace_batch(const or_medium *m, const double *depth, const double *ice,
                       const double *txh, const double *dist, size_t n, double *out10,
                       int nthreads);

#ifdef __cplusplus
}
#endif
#endif

/* ---- Table lookup: GetHorizontalDistanceToIntersectionPoint_Table ----------
 * .cc:1305-1462 with GetParValues :1172-1302, FindClosestAirTxHeight :1033-1126,
 * FindClosestTHD :1128-1169, oneDLinearInterpolation :992-995.  The table is one antenna's
 * AllTableAllAntData[ant] (11 float columns of n entries); the grid globals are those of the
 * LAST MakeRayTracingTable call (the reference reads them, .cc:1035). */
typedef struct or_lookup_table {
  const float *col[11];
  long n;
  double LoopStopHeight, HeightStepSize;
  int TotalHeightSteps, TotalAngleSteps;
} or_lookup_table;
/* flags of one lookup */
enum {
  OR_LK_FALLBACK = 1, /* the minimizer fallback ran (.cc:1418-1420, with its x100 argument quirk) */
  OR_LK_UNPINNED = 2  /* outputs read uninitialised / out-of-range memory in the reference */
};
/* outs[9] in the order of the reference's reference arguments; returns CheckSolution. */
int or_table_lookup(const or_medium *m, const or_lookup_table *t, double src_cm, double dist_cm,
                    double depth_cm, double ice_cm, double outs[9], int *flags);
/* n queries (cm) against one table; out: 9 columns of stride ld; ok/flags per query. */
void or_table_lookup_batch(const or_medium *m, const or_lookup_table *t, const double *src_cm,
                           const double *dist_cm, const double *depth_cm, double ice_cm, size_t n,
                           double *out, size_t ld, unsigned char *ok, unsigned char *flags,
                           int nthreads);

/* ---- SingleRayAirIceRefraction CLI (cfg1; SURVEY §8 a19 + the f4 path sampler) ----------
 * SingleRayAirIceRefraction.C:33-299 over RayTracingFunctions.cc (same medium, pi 3.1415927):
 * forward trace of one launch angle (the layer loop :100-154, GetIcePropagationPar :166) and
 * the x(z) path at 1 m steps written to RayPathinAirnIce.txt (:226-299).  Inputs are the
 * values after the CLI's clamps (:40-51); antenna depth is POSITIVE in ice (:166). */
typedef struct or_single_ray {
  int skip_above, skip_below, n_layers; /* n_layers = MaxLayers - SkipAbove - SkipBelow */
  double thd_air;                       /* "Total horizontal distance ..." (:157) */
  double L;                             /* Lvalue = layerLs[*] = LvalueIce */
  double inc_ice;                       /* IncidentAngleonIce, deg (:156) */
  double thd_ice, recv_ice, t_ice;      /* GetIcePropagationPar outputs (:166-170) */
  long n_air, n_ice;                    /* path samples in air / ice */
} or_single_ray;
/* x/z (nullable): capacity cap >= n_air + n_ice samples, in file order (ipoints). */
/* RayTracingFunctions:: scalar layer in its own layouts; op as AIRICE_RTF_*; returns outputs. */
int or_rtf_eval(const or_medium *m, int op, const double *args, double *out);

int or_single_ray_trace(const or_medium *m, double depth, double launch_deg, double txh,
                        double ice, or_single_ray *out, double *x, double *z, long cap);
