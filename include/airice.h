/*
 * airice.h -- C-ABI of libairice.so, the MI355X (gfx950) implementation of the
 * uzairlatif90/AirIceRayTracing hot path:
 *   - MultiRayAirIceRefraction table generation  (MakeRayTracingTable,
 *     MultiRayAirIceRefraction.cc:2019-2158, one ray = GetRayTracingSolutions .cc:1796-2017)
 *   - per-(Tx,Rx) launch-angle root finding      (Air2IceRayTracing .cc:1464-1616 and the
 *     CoREAS entry GetHorizontalDistanceToIntersectionPoint .cc:945-989)
 *   - the pythonwrapper ctypes surface           (Py_TraceIceToAir, pythonwrapper/TraceIceToAir.C:75-79)
 *
 * Plain C types only (no HIP / torch types).  Device pointers are hipMalloc'd (or
 * torch CUDA tensors' data_ptr) and `stream` is a hipStream_t passed as void*
 * (NULL = default stream).  All *_launch entry points are stream-ordered and
 * asynchronous; *_host entry points copy, launch and synchronise.
 *
 * Errors: every int-returning function returns AIRICE_OK (0) or a negative
 * AIRICE_E* code; airice_last_error() gives a message.  Numerical failure modes
 * follow the reference (NaN propagation, -1000 / zeroed outputs), see DESIGN.md.
 *
 * Thread safety: the reference library is not reentrant (namespace statics,
 * MultiRayAirIceRefraction.h:33-81).  Here the medium is an explicit value
 * (airice_medium) and every batch entry point is reentrant.
 */
#ifndef AIRICE_H
#define AIRICE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AIRICE_OK 0
#define AIRICE_EINVAL (-1)
#define AIRICE_EIO (-2)
#define AIRICE_EHIP (-3)
#define AIRICE_ENOMEM (-4)

/* Variant of the reference namespace whose numerics are reproduced. */
#define AIRICE_VARIANT_MULTIRAY 0  /* MultiRayAirIceRefraction:: (pi = 3.1415927, .h:29) */
#define AIRICE_VARIANT_PYWRAPPER 1 /* AirIceRayTracing::        (pi = 4*atan(1), pythonwrapper .h:25) */

/* Per-query solve status bits (GSL 2.x bisection semantics). */
/* AIRICE_SOLVE_NONFINITE_END: f(lo) or f(hi) is non-finite, so gsl_root_fsolver_set returns before
 * storing f_lower/f_upper and the reference's next gsl_root_fsolver_iterate reads uninitialised
 * malloc memory.  The reference's result on such a row is undefined; this
 * library (and the oracle) model a zero-filled solver state, which is deterministic but NOT what
 * real GSL returns -- a consumer comparing against GSL must mask these rows (about 0.7 % of the
 * cfg3 distribution), as the parity tests do.  AIRICE_SOLVE_BAD_BRACKET and
 * AIRICE_SOLVE_NO_AIR_LAYER rows are undefined in the reference in the same sense. */
#define AIRICE_SOLVE_NONFINITE_END 1 /* f(lo) or f(hi) non-finite: reference reads uninitialised GSL state */
#define AIRICE_SOLVE_BAD_BRACKET 2   /* lo > hi: gsl_root_fsolver_set fails */
#define AIRICE_SOLVE_STALE_MID 4     /* a bisection midpoint gave non-finite f: root frozen */
#define AIRICE_SOLVE_PROBED 8        /* bracket-probe loop ran (.cc:1490-1511) */
#define AIRICE_SOLVE_MAXITER 16      /* 40 iterations, interval test never passed */
#define AIRICE_SOLVE_NO_AIR_LAYER 32 /* no air layer between Tx and the ice */

/* Medium: the GDAS layered atmosphere reduced to its run-time parameters plus the
 * ice model.  Filled by airice_atmosphere_* (readATMpar .cc:24-71, readnhFromFile
 * .cc:73-147, MakeAtmosphere .cc:920-942, FillInAirRefractiveIndex .cc:193-213). */
typedef struct airice_medium {
  double atmlay_cm[5];   /* ATMLAY (cm); [4] forced to 1.5e7 (.cc:66) */
  double abc[5][3];      /* mass-overburden a,b,c rows; abc[4]=abc[3] (.cc:62-64) */
  double B_air[5];       /* n(h) = A_air + B_air[l]*exp(-C_air[l]*h) */
  double C_air[5];
  double N0;             /* natural cubic spline of n(h) at h=0 (.cc:203) */
  int32_t max_layers;    /* MaxLayers (.cc:142) */
  int32_t n_points;      /* knots in the flattened profile */
  double A_air;          /* 1.0 (.h:99) */
  double A_ice, B_ice, C_ice; /* 1.78, -0.43, 0.0132 (.h:64-66) */
  double pi;             /* variant constant */
  double h_top;          /* h_data.back().back(): last tabulated height, m (the Tx clamp of
                            SingleRayAirIceRefraction.C:40-45) */
  int32_t constant_air_index; /* pythonwrapper AirIceRayTracing::UseConstantRefractiveIndex
                                 (.h:54, default 0): honoured by AIRICE_VARIANT_PYWRAPPER only --
                                 GetB_air = 0, GetC_air = 1e-9, Getnz_air = A_const (.cc:173-238)
                                 and the launch bracket [90, thR] without the probe (.cc:955-982) */
  int32_t reserved_;
  double A_const;        /* pythonwrapper .h:72 (1.00) */
} airice_medium;

/* MakeRayTracingTable grid (.cc:12-21 globals, .cc:2019-2061 set-up). */
typedef struct airice_grid {
  double start_height;   /* LoopStartHeight, m (100000, .cc:2044) */
  double stop_height;    /* LoopStopHeight, m: ice, or ice+depth when Rx is in air */
  double height_step;    /* HeightStepSize, m (10) */
  int32_t height_steps;  /* TotalHeightSteps */
  double start_angle;    /* LoopStartAngle, deg (90.1) */
  double stop_angle;     /* LoopStopAngle, deg (180) */
  double angle_step;     /* AngleStepSize, deg (0.1) */
  int32_t angle_steps;   /* TotalAngleSteps */
  double depth_m;        /* AntennaDepth, m (negative = in ice) */
  double ice_m;          /* IceLayerHeight, m */
  int32_t in_ice;        /* AntennaDepth < 0 */
  int32_t table_rows;    /* rows the table holds: the reference skips every row whose Tx height
                            start_height - height_step*row is not > 0 (.cc:2082), a suffix of the
                            height_steps rows, so the table is table_rows x angle_steps entries
                            (height_steps itself stays TotalHeightSteps, which the lookup reads) */
} airice_grid;

#define AIRICE_TABLE_COLUMNS 11 /* float columns of AllTableAllAntData (.cc:2101-2111) */
#define AIRICE_RAY_FIELDS 18    /* GetRayTracingSolutions dummy[0..17] (.cc:1999-2016) */
#define AIRICE_SOLVE_FIELDS 17  /* Air2IceRayTracing dummy[0..16] (.cc:1597-1614) */
#define AIRICE_PYSOLVE_FIELDS 15 /* AirIceRayTracing::Air2IceRayTracing dummy[0..14] (pythonwrapper .cc:1070-1084) */
#define AIRICE_HDTIP_FIELDS 9   /* GetHorizontalDistanceToIntersectionPoint outputs (.cc:963-972) */

const char *airice_last_error(void);
const char *airice_version(void);

/* --- medium (host) ------------------------------------------------------ */
/* Parse a GDAS Atmosphere.dat from a file (replaces MakeAtmosphere(), .cc:920). */
int airice_atmosphere_load(const char *path, int variant, airice_medium *out);
/* Parse from an in-memory text image of the same file. */
int airice_atmosphere_parse(const char *text, size_t len, int variant, airice_medium *out);
/* n(z) of the medium (Getnz_air .cc:259, Getnz_ice .cc:188), host side. */
double airice_nz_air(const airice_medium *m, double z);
double airice_nz_ice(const airice_medium *m, double z);

/* --- table (MakeRayTracingTable) ---------------------------------------- */
/* Grid set-up exactly as .cc:2019-2061 (depth/ice in cm as the reference takes them). */
int airice_grid_init(airice_grid *g, double antenna_depth_cm, double ice_height_cm,
                     double height_step_m, double start_angle_deg, double stop_angle_deg,
                     double angle_step_deg);
/* Trace rows [row_begin, row_begin+row_count) x all angles of the grid (rows at or past
 * table_rows are skipped, as the reference skips Tx heights <= 0).
 * d_table: 11 float columns, column c of ray r at d_table[c*ld + r - row_begin*angle_steps]
 * (the AllTableAllAntData[ant][c][r] layout).  d_full (nullable): 18 double columns,
 * same indexing (GetRayTracingSolutions dummy[] for parity checks). */
int airice_table_launch(const airice_medium *m, const airice_grid *g, int32_t row_begin,
                        int32_t row_count, float *d_table, double *d_full, size_t ld,
                        void *stream);
/* Several antennas' tables in ONE launch (one grid over every antenna's rows; the reference's
 * per-antenna loop RunMultiRayCode.C:29-52 calls MakeRayTracingTable once per antenna): grids[a]
 * from airice_grid_init for antenna a (same angle grid for all), d_tables[a] its 11 float columns
 * with column stride lds[a] >= grids[a].table_rows * angle_steps.  Bit-identical to one
 * airice_table_launch per antenna; at most 32 antennas. */
int airice_table_launch_multi(const airice_medium *m, const airice_grid *grids, int32_t n_grids,
                              float *const *d_tables, const size_t *lds, void *stream);
int airice_table_host(const airice_medium *m, const airice_grid *g, int32_t row_begin,
                      int32_t row_count, float *h_table, double *h_full, size_t ld);

/* --- single forward ray (GetRayTracingSolutions) on the device ---------- */
/* n rays with per-ray (launch_deg, txh_m); ice/depth/in_ice uniform; out: 18 double columns. */
int airice_rays_launch(const airice_medium *m, const double *d_launch_deg, const double *d_txh,
                       double ice_h_m, double depth_m, int32_t in_ice, size_t n, double *d_out,
                       size_t ld, void *stream);

/* The same rays on the host (CPU), from the same source as the device kernels with the host's
 * correctly rounded sqrt and quotients (within ~1 ulp of the device's): the one-query
 * GetRayTracingSolutions of the C++ drop-in runs here, ~1 us against a ~10 us kernel round trip.
 * Host arrays; out: 18 double columns, stride ld. */
int airice_rays_host(const airice_medium *m, const double *launch_deg, const double *txh,
                     double ice_h_m, double depth_m, int32_t in_ice, size_t n, double *out,
                     size_t ld);

/* Where one-query calls run: AIRICE_SCALAR_HOST (default: the calling CPU thread, from the same
 * __host__ __device__ source as the kernels, with the host's correctly rounded sqrt and quotients,
 * so within about an ulp of the same query inside a GPU batch) or AIRICE_SCALAR_DEVICE (a
 * one-wave GPU kernel per call, bit-identical to the batch).  The mode covers every one-query
 * call: GetRayTracingSolutions and the ray layer of the C++ drop-ins (airice_rtf_eval / _variant:
 * RayTracingFunctions::, MultiRayAirIceRefraction:: and AirIceRayTracing:: fDnfR ...
 * MinimizeforLaunchAngle), the one-query solves (Air2IceRayTracing, the CoREAS entry,
 * Py_TraceIceToAir, the _Table lookup's minimizer fallback) and airice_solve_host /
 * airice_trace_ice_to_air_host calls with n == 1.  The environment variable AIRICE_SCALAR=device
 * selects the device at start.  Returns the previous mode; any other value only queries it.
 * Batch entry points (n > 1 and every *_launch) always run on the GPU; airice_rays_host always
 * runs on the host. */
#define AIRICE_SCALAR_HOST 0
#define AIRICE_SCALAR_DEVICE 1
int airice_scalar_mode(int mode);

/* --- minimizer (Air2IceRayTracing) --------------------------------------- */
/* Batched launch-angle solve.  Inputs in metres: Tx height, horizontal distance, Rx
 * depth (negative = below the ice surface); ice height uniform.  d_straight_angle is
 * Air2IceRayTracing's StraightAngle argument (.cc:1464) in degrees; when NULL it is
 * formed per query as GetHorizontalDistanceToIntersectionPoint does (.cc:952-958).
 * d_out: AIRICE_SOLVE_FIELDS (MultiRay) or AIRICE_PYSOLVE_FIELDS (pythonwrapper)
 * double columns, stride ld.  d_status (nullable): AIRICE_SOLVE_* bits. */
int airice_solve_launch(const airice_medium *m, int variant, double ice_h_m,
                        const double *d_txh, const double *d_dist, const double *d_depth,
                        const double *d_straight_angle, size_t n, double *d_out, size_t ld,
                        uint8_t *d_status, void *stream);
int airice_solve_host(const airice_medium *m, int variant, double ice_h_m, const double *txh,
                      const double *dist, const double *depth, const double *straight_angle,
                      size_t n, double *out, size_t ld, uint8_t *status);

/* CoREAS entry, batched: GetHorizontalDistanceToIntersectionPoint (.cc:945-989) with cm
 * inputs; d_out: 9 double columns (opticalPathLengthInIce, opticalPathLengthInAir,
 * geometricalPathLengthInIce, geometricalPathLengthInAir, launchAngle [rad],
 * horizontalDistanceToIntersectionPoint, transmissionCoefficientS,
 * transmissionCoefficientP, RecievedAngleInIce [rad]); d_ok: the returned bool. */
int airice_hdtip_launch(const airice_medium *m, const double *d_src_cm, const double *d_dist_cm,
                        const double *d_depth_cm, double ice_cm, size_t n, double *d_out,
                        size_t ld, uint8_t *d_ok, void *stream);

/* --- table lookup (GetHorizontalDistanceToIntersectionPoint_Table) -------- */
/* One antenna's table resident in HBM (the AllTableAllAntData[ant] a MakeRayTracingTable /
 * airice_table_launch produced) plus the grid globals the reference reads at lookup time
 * (LoopStopHeight, HeightStepSize, TotalHeightSteps, TotalAngleSteps of the LAST table made,
 * .cc:1035-1039). */
typedef struct airice_lookup_table {
  const float *table;         /* device: column c of entry i at table[c*ld + i] */
  size_t ld;                  /* column stride in floats */
  size_t n_entries;           /* AllTableAllAntData[ant][0].size() */
  double loop_stop_height;    /* m */
  double height_step;         /* m */
  int32_t total_height_steps;
  int32_t total_angle_steps;
  const float *entries;       /* optional device copy from airice_lookup_pack (NULL: the lookup
                                 reads the columns only); same values, fewer cache lines */
} airice_lookup_table;

/* The packed copy (pack format 2, library 0.2; format 1 of 0.1.x had 32-float pair records and
 * no angle vector -- a buffer sized for it is too small and airice_lookup_pack refuses it):
 *  - pair records: record i holds columns 2, 3, 5, 6, 7, 8, 9, 10 of entry i (floats 0-7) and of
 *    entry i + 1 (floats 8-15; NaN for the last entry): 64 B, one fabric request when the array
 *    is 64-byte aligned.  The lookup interpolates between entries i and i + 1 (FindClosestTHD's
 *    index1, index2), so each table row it visits costs it one record; the THD values at the pair
 *    (column 1) come from its own search, the launch angles (column 4) from the angle vector;
 *  - row records, from float AIRICE_LOOKUP_ROWS_OFFSET(n_entries) on (128-byte aligned), one per
 *    full table row (n_entries / total_angle_steps rows): the row's FindClosestAirTxHeight span,
 *    the table values the lookup reads at its ends and the THD values of the first four
 *    FindClosestTHD bisection steps on both interpolation heights' spans (two 128-byte lines);
 *  - the angle vector: column 4 of the first row (total_angle_steps floats, padded to 4), then one
 *    int32 word: 1 when every row's column 4 equals it bit for bit (a MakeRayTracingTable table:
 *    the launch angle is the grid's, .cc:2084-2105), else 0 and the lookup reads column 4. */
#define AIRICE_LOOKUP_ENTRY_FLOATS 16
#define AIRICE_LOOKUP_ROW_FLOATS 64
#define AIRICE_LOOKUP_ROWS_OFFSET(n_entries) \
  (((size_t)(n_entries) * AIRICE_LOOKUP_ENTRY_FLOATS + 31) / 32 * 32)
/* Floats of the whole packed copy. */
#define AIRICE_LOOKUP_PACK_FLOATS(n_entries, angle_steps)                          \
  (AIRICE_LOOKUP_ROWS_OFFSET(n_entries) +                                         \
   ((size_t)(n_entries) / (size_t)(angle_steps)) * AIRICE_LOOKUP_ROW_FLOATS +     \
   ((size_t)(angle_steps) + 3) / 4 * 4 + 4)
/* The same, as a call (0 when n_entries or total_angle_steps is < 1). */
size_t airice_lookup_pack_floats(size_t n_entries, int32_t total_angle_steps);

/* Pack one antenna's table for the lookup into d_entries: capacity_floats (at least
 * AIRICE_LOOKUP_PACK_FLOATS(n_entries, total_angle_steps), else AIRICE_EINVAL and nothing is
 * written) device floats, 16-byte aligned (64-byte for one request per pair record).  The lookup
 * then reads the interpolated parameters of both entries of a pair from one record instead of 10
 * columns ld floats apart; results are identical.  Stream-ordered; run once per table, then set
 * t->entries = d_entries. */
int airice_lookup_pack(const airice_lookup_table *t, float *d_entries, size_t capacity_floats,
                       void *stream);

#define AIRICE_LOOKUP_FALLBACK 1 /* the minimizer fallback ran (.cc:1418-1420) */
#define AIRICE_LOOKUP_UNPINNED 2 /* the reference reads uninitialised/out-of-range memory here:
                                    such slots are returned as 0 / NaN */

/* Batched GetHorizontalDistanceToIntersectionPoint_Table (.cc:1305-1462) for one antenna
 * (AntennaNumber already resolved by the caller, .cc:1348-1352): cm inputs, ice height
 * uniform; d_out: the 9 double columns of airice_hdtip_launch, d_ok: the returned bool,
 * d_flags (required): AIRICE_LOOKUP_* bits.  Lanes hitting the reference's one-sided
 * extrapolation case run its minimizer fallback on the device, with the reference's
 * argument handling (cm values scaled by 100 once more, optical/geometric slots swapped). */
int airice_table_lookup_launch(const airice_medium *m, const airice_lookup_table *t,
                               const double *d_src_cm, const double *d_dist_cm,
                               const double *d_depth_cm, double ice_cm, size_t n,
                               double *d_out, size_t ld, uint8_t *d_ok, uint8_t *d_flags,
                               void *stream);

/* --- single ray + path sampler (SingleRayAirIceRefraction, BASELINE cfg1) ---------------- */
/* SingleRayAirIceRefraction.C:33-299 over RayTracingFunctions.cc: inputs are the CLI's values
 * after its clamps (Tx <= h_top, launch > 90, .C:40-51), metres/degrees, antenna depth
 * POSITIVE below the ice surface (.C:166).  Path samples are the lines of
 * RayPathinAirnIce.txt in order: x (m) and height z (m). */
typedef struct airice_single_ray_info {
  int32_t skip_above, skip_below; /* SkipLayersAbove / SkipLayersBelow (.C:60-86) */
  int32_t n_layers;               /* MaxLayers - SkipLayersAbove - SkipLayersBelow (.C:226) */
  int32_t pad_;
  int64_t n_air, n_ice;           /* path samples in air (.C:247) and ice (.C:292) */
} airice_single_ray_info;
/* summary: total horizontal distance in air (.C:157), L, incident angle on the ice (deg),
 * horizontal distance / receive angle (deg) / propagation time (s) in ice (.C:167-170) */
#define AIRICE_SINGLE_RAY_FIELDS 6
#define AIRICE_SINGLE_RAY_WORK 32 /* doubles of d_summary: the summary, then sampler constants */
int airice_single_ray_plan(const airice_medium *m, double antenna_depth_m, double launch_deg,
                           double txh_m, double ice_m, airice_single_ray_info *info);
/* d_summary: AIRICE_SINGLE_RAY_WORK doubles (summary in the first AIRICE_SINGLE_RAY_FIELDS);
 * d_x/d_z (nullable together): cap >= n_air + n_ice */
int airice_single_ray_launch(const airice_medium *m, double antenna_depth_m, double launch_deg,
                             double txh_m, double ice_m, double *d_summary, double *d_x,
                             double *d_z, size_t cap, void *stream);
int airice_single_ray_host(const airice_medium *m, double antenna_depth_m, double launch_deg,
                           double txh_m, double ice_m, double *summary, double *x, double *z,
                           size_t cap);

/* pythonwrapper TraceIceToAir, batched: per-query (depth, ice, txh, dist) metres ->
 * ArrayParameters[10] rows (TraceIceToAir.C:46-68), row-major n x 10. */
int airice_trace_ice_to_air_launch(const airice_medium *m, const double *d_depth,
                                   const double *d_ice, const double *d_txh,
                                   const double *d_dist, size_t n, double *d_out10,
                                   void *stream);
int airice_trace_ice_to_air_host(const airice_medium *m, const double *depth, const double *ice,
                                 const double *txh, const double *dist, size_t n, double *out10);

/* Drop-in for the reference ctypes symbol (TraceIceToAir.C:75-79): the C++ TraceIceToAir of
 * include/AirIceRayTracing.h, which reads "Atmosphere.dat" from the working directory like the
 * reference (parsed once while the file is unchanged; falls back to $AIRICE_ATMOSPHERE), then
 * solves the one query where airice_scalar_mode says: the calling thread by default, a one-wave
 * GPU kernel with AIRICE_SCALAR=device.  Batches: airice_trace_ice_to_air_launch. */
void Py_TraceIceToAir(double AntennaDepth, double IceLayerHeight, double AirTxHeight,
                      double HorizontalDistance, double ArrayParameters[10]);

/* --- RayTracingFunctions:: scalar layer (RayTracingFunctions.cc, the cfg1 CLI's library) --- */
/* One call evaluated with the reference's expressions (pi 3.1415927) on the host, or on the
 * device (airice_scalar_mode); host arguments and outputs, synchronous.  For the
 * RayTracingFunctions.h drop-in (include/RayTracingFunctions.h); batches belong on the table /
 * solve / single-ray paths. */
#define AIRICE_RTF_HIT_POINT 0        /* GetLayerHitPointPar (.cc:399-527)
                                         args {n_layer1, RxDepth, TxDepth, IncidentAng, AirOrIce}
                                         -> {THD, ReceiveAngle deg, L, time s} */
#define AIRICE_RTF_OPTICAL_PATH 1     /* GetRayOpticalPath (.cc:349-369)
                                         args {A, RxDepth, TxDepth, Lvalue, AirOrIce} -> {x} */
#define AIRICE_RTF_PROPAGATION_TIME 2 /* GetRayPropagationTime (.cc:371-397), args as above */
#define AIRICE_RTF_AIR_PROPAGATION 3  /* GetAirPropagationPar (.cc:529-659)
                                         args {LaunchAngle, AirTxHeight, IceLayerHeight}
                                         -> 4 x MaxLayers {THD, Recv, L, t} + count */
#define AIRICE_RTF_ICE_PROPAGATION 4  /* GetIcePropagationPar (.cc:661-681) args {IncidentAngle,
                                         IceLayerHeight, AntennaDepth, Lvalue} -> {THD, Recv, L, t} */
#define AIRICE_RTF_FDNFR 5            /* fDnfR (.cc:293-303) args {x, a, b, c, l} -> {value} */
#define AIRICE_RTF_FTIMED 6           /* ftimeD (.cc:328-347) args {x, a, b, c, speedc, l,
                                         airorice} -> {value} */
#define AIRICE_RTF_MIN_LAUNCH 7       /* MinimizeforLaunchAngle (.cc:683-731) args {x, airtxheight,
                                         icelayerheight, antennadepth, horizontaldistance} */
#define AIRICE_RTF_AIR2ICE 8          /* the Air2IceRayTracing CLI's solve (Air2IceRayTracing.C:56-185):
                                         args {AirTxHeight, HorizontalDistance, IceLayerHeight,
                                         AntennaDepth (> 0 in ice)} -> AIRICE_RTF_AIR2ICE_FIELDS:
                                         launch-angle bracket and its probe, GSL-Brent root of
                                         MinimizeforLaunchAngle (FindFunctionRoot, .cc:256-290,
                                         max_iter 20, tolerance 1e-9), air and ice results */
#define AIRICE_RTF_AIR2ICE_FIELDS 16  /* {startangle, endangle, LaunchAngleAir, THD_air,
                                         IncidentAngleonIce, Lvalue, t_air ns, THD_ice,
                                         IncidentAngleonAntenna, t_ice ns, THD, t ns,
                                         status (AIRICE_SOLVE_* bits), Brent iterations,
                                         probe steps, filled air layers} */
/* MultiRayAirIceRefraction:: forms of the same layer (MultiRayAirIceRefraction.cc:377-917, the
 * MultiRayAirIceRefraction.h drop-in): 5-wide outputs {THD, ReceiveAngle deg, L, time s,
 * geometric path}.  fDnfR, ftimeD and GetRayPropagationTime are the AIRICE_RTF_ ops above
 * (identical expressions), GetRayHorizontalPath is AIRICE_RTF_OPTICAL_PATH. */
#define AIRICE_MR_FPATHD 9            /* fpathD (.cc:434-447) args {x, a, b, c, speedc, l} */
#define AIRICE_MR_GEOMETRIC_PATH 10   /* GetRayGeometricPath (.cc:494-513)
                                         args {A, RxDepth, TxDepth, Lvalue, AirOrIce} */
#define AIRICE_MR_HIT_POINT 11        /* GetLayerHitPointPar (.cc:521-646)
                                         args {n_layer1, RxDepth, TxDepth, IncidentAng, AirOrIce} */
#define AIRICE_MR_AIR_PROPAGATION 12  /* GetAirPropagationPar (.cc:661-804) args {LaunchAngle,
                                         AirTxHeight, IceLayerHeight} -> 5 x MaxLayers + 2,
                                         filled-layer count at [5*MaxLayers+1] */
#define AIRICE_MR_ICE_PROPAGATION 13  /* GetIcePropagationPar (.cc:807-869) args {IncidentAngleonIce,
                                         IceLayerHeight, AntennaDepth, Lvalue} -> 5 */
#define AIRICE_MR_MIN_LAUNCH 14       /* MinimizeforLaunchAngle (.cc:873-917) args {x, airtxheight,
                                         icelayerheight, antennadepth, horizontaldistance} */
/* Outputs written for op (4 x max_layers + 1 for AIR_PROPAGATION, 5 x max_layers + 2 for
 * MR_AIR_PROPAGATION), or -1 for an unknown op. */
int airice_rtf_outputs(int op, int max_layers);
int airice_rtf_eval(const airice_medium *m, int op, const double *args, size_t n_args,
                    double *out, size_t n_out);
/* The same ops with the numerics of another reference namespace: AIRICE_VARIANT_PYWRAPPER gives the
 * pythonwrapper's AirIceRayTracing:: ray layer (pythonwrapper/AirIceRayTracing.cc:356-857, the
 * AIRICE_MR_* / FDNFR / FTIMED / OPTICAL_PATH / PROPAGATION_TIME ops with pi = 4*atan(1) and its
 * UseConstantRefractiveIndex medium); airice_rtf_eval is AIRICE_VARIANT_MULTIRAY. */
int airice_rtf_eval_variant(const airice_medium *m, int variant, int op, const double *args,
                            size_t n_args, double *out, size_t n_out);

/* Device bookkeeping (thin wrappers so ctypes callers need no HIP runtime binding). */
int airice_device_count(int *count);
int airice_set_device(int device);
int airice_malloc(void **ptr, size_t bytes);
int airice_free(void *ptr);
int airice_memcpy_h2d(void *dst, const void *src, size_t bytes);
int airice_memcpy_d2h(void *dst, const void *src, size_t bytes);
int airice_synchronize(void);

/* Host assembly of tables (MakeRayTracingTable keeps AllTableAllAntData in host memory,
 * .cc:2101-2136): copy n_rays entries of the 11 float columns of a device table (column stride
 * d_ld) into a host table (column stride h_ld), stream-ordered (one 2-D DMA: hipMemcpy2DAsync).
 * h_table should be pinned (hipHostMalloc'd or registered with airice_host_register) for the copy
 * to be asynchronous at full PCIe rate.  A rank of a sharded build copies its row slab to
 * h_table + (first ray of the slab). */
int airice_table_to_host(const float *d_table, size_t d_ld, size_t n_rays, float *h_table,
                         size_t h_ld, void *stream);
/* Page-lock an existing host range for DMA (hipHostRegister, portable) / undo it. */
int airice_host_register(void *ptr, size_t bytes);
int airice_host_unregister(void *ptr);

/* --- table persistence (no reference counterpart: the reference keeps
 * AllTableAllAntData in memory only, .cc:2101-2136) -------------------------------------------
 * One antenna's host table in a file: a 512-byte little-endian header (magic "AIRTBL01", the
 * medium and grid it was traced with, the entry count, a 64-bit checksum of the column bytes),
 * then the 11 float32 columns of n_rays entries each, column after column.  Host-only (no GPU
 * needed); a device table goes through airice_table_to_host first. */
#define AIRICE_TABLE_FILE_HEADER 512
typedef struct airice_table_file_info {
  airice_medium medium; /* the medium the table was traced in */
  airice_grid grid;     /* its grid; n_rays = table_rows x angle_steps for a whole table */
  uint64_t n_rays;      /* entries per column */
  uint64_t checksum;    /* of the 11 columns' bytes (airice_table_checksum) */
} airice_table_file_info;
/* 64-bit checksum of n_rays entries of the 11 columns (column stride ld). */
uint64_t airice_table_checksum(const float *h_table, size_t ld, size_t n_rays);
int airice_table_save(const char *path, const airice_medium *m, const airice_grid *g,
                      const float *h_table, size_t ld, size_t n_rays);
/* Header of a table file (validated: magic, version, sizes against the file length). */
int airice_table_file_read_info(const char *path, airice_table_file_info *info);
/* Load a table file into h_table (column stride ld >= the file's n_rays), verifying its checksum.
 * expect (nullable): the medium the caller traces with -- a file traced in another medium (any
 * parsed field differs) is rejected with AIRICE_EINVAL.  info (nullable) receives the header. */
int airice_table_load(const char *path, const airice_medium *expect, float *h_table, size_t ld,
                      airice_table_file_info *info);

/* Kernel timing (bench.py's roofline legs; no reference counterpart).  When on, each launch
 * of a timed kernel is bracketed by a hipEvent pair on its own stream.  Names:
 * "table_kernel", "roots_kernel" (roots_kernel / roots_sorted_kernel, the minimizer's root
 * finder), "group_passes" (the batch-wide grouping passes), "out_kernel" (solve_out /
 * hdtip_out / trace_out), "lookup_kernel".  airice_kernel_time waits for the recorded pairs
 * and returns their summed duration and count; reset != 0 clears them. */
int airice_kernel_timing(int on);
int airice_kernel_time(const char *name, double *total_ms, int64_t *launches, int reset);

/* Launch counters (no reference counterpart; always on, one atomic increment per launch): how
 * many times a kernel was launched in this process since the last reset, so a test can prove the
 * device path it checks really ran.  Names: "table_kernel", "rays_kernel", "scalar_ray_kernel",
 * "roots_kernel" (roots_kernel / roots_sorted_kernel), "scalar_solve_kernel" (the one-query
 * minimizer entry points in AIRICE_SCALAR_DEVICE mode), "out_kernel", "lookup_kernel",
 * "rtf_kernel" (ray layer and the GSL-Brent search), "single_ray_kernel", "path_kernel".
 * AIRICE_LAUNCH_REPORT=1 in the environment prints every count to stderr when the library
 * unloads. */
int airice_launch_count(const char *name, int64_t *count, int reset);

/* The table launch's per-grid caches on the current device (no reference counterpart; tests and
 * diagnostics).  out[0..2]: row-constant keys seen, of them filled (device buffer resident),
 * pinned (used by a launch captured into a graph); out[3..5]: the same for the start-angle
 * sines.  A grid's first launch only records its key; the second fills the buffers, stream-ordered
 * (INTEGRATION.md §5). */
int airice_table_cache_stats(int out[6]);

#ifdef __cplusplus
}
#endif
#endif /* AIRICE_H */
