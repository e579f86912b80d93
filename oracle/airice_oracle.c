/*
 * airice_oracle.c -- TEST INFRASTRUCTURE ONLY (see airice_oracle.h).
 *
 * Plain-C restatement of the reference hot path, written from the reference's
 * behaviour (file:line cited per function).  Faithful mode: each reference
 * function is a function here, with the same per-call layer scans, the same
 * libm calls and the same expression order (pow(x,2) is written x*x, which is
 * what g++ -O2 folds it to).  Build: oracle/Makefile (gcc -O2 -ffp-contract=off).
 *
 * Third-party algorithms restated (GNU GSL, absent from this image; the
 * reference pins "2.4 is verified", README.md:37, and links libgsl.so.23/.27):
 *   - gsl_interp_cspline natural cubic spline (interpolation/cspline.c) with
 *     gsl_linalg_solve_symm_tridiag (linalg/tridiag.c), evaluated once for N0;
 *   - gsl_root_fsolver_bisection + gsl_root_test_interval
 *     (roots/bisection.c, roots/convergence.c, roots/fsolver.c).
 */
#include "airice_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static const double SPEEDC = 299792458.0; /* MultiRayAirIceRefraction.h:30 */

/* ------------------------------------------------------------------------- */
/* iostream emulation for the GDAS parser (std::getline / operator>> / ignore) */
/* ------------------------------------------------------------------------- */
typedef struct {
  const char *p, *end;
  int fail;
} or_stream;

static int st_getline(or_stream *s) {
  if (s->fail) return 0;
  if (s->p >= s->end) { s->fail = 1; return 0; }
  while (s->p < s->end && *s->p != '\n') s->p++;
  if (s->p < s->end) s->p++; /* consume delimiter */
  return 1;
}

static void st_ignore(or_stream *s, int n, char delim) {
  if (s->fail) return;
  for (int i = 0; i < n && s->p < s->end; i++) {
    char c = *s->p++;
    if (c == delim) break;
  }
}

/* operator>>(double&): skip ws; at EOF -> fail, value unchanged (sentry fails). */
static void st_read_double(or_stream *s, double *v) {
  if (s->fail) return;
  while (s->p < s->end && (*s->p == ' ' || *s->p == '\t' || *s->p == '\n' || *s->p == '\r'
                           || *s->p == '\v' || *s->p == '\f'))
    s->p++;
  if (s->p >= s->end) { s->fail = 1; return; }
  char buf[64];
  size_t k = 0;
  const char *q = s->p;
  while (q < s->end && k < sizeof(buf) - 1 && !(*q == ' ' || *q == '\t' || *q == '\n' || *q == '\r'))
    buf[k++] = *q++;
  buf[k] = 0;
  char *ep = NULL;
  double x = strtod(buf, &ep);
  if (ep == buf) { *v = 0.0; s->fail = 1; return; }
  s->p += (ep - buf);
  *v = x;
}

/* ------------------------------------------------------------------------- */
/* GSL natural cubic spline (cspline_init natural BC + solve_symm_tridiag +    */
/* cspline_eval), restated.                                                    */
/* ------------------------------------------------------------------------- */
double or_spline_eval_at(const double *xa, const double *ya, int size, double x) {
  const int max_index = size - 1;
  const int sys_size = max_index - 1;
  double *c = (double *)calloc((size_t)size, sizeof(double));
  double *g = (double *)malloc(sizeof(double) * (size_t)sys_size);
  double *diag = (double *)malloc(sizeof(double) * (size_t)sys_size);
  double *offdiag = (double *)malloc(sizeof(double) * (size_t)sys_size);
  for (int i = 0; i < sys_size; i++) {
    const double h_i = xa[i + 1] - xa[i];
    const double h_ip1 = xa[i + 2] - xa[i + 1];
    const double ydiff_i = ya[i + 1] - ya[i];
    const double ydiff_ip1 = ya[i + 2] - ya[i + 1];
    const double g_i = (h_i != 0.0) ? 1.0 / h_i : 0.0;
    const double g_ip1 = (h_ip1 != 0.0) ? 1.0 / h_ip1 : 0.0;
    offdiag[i] = h_ip1;
    diag[i] = 2.0 * (h_ip1 + h_i);
    g[i] = 3.0 * (ydiff_ip1 * g_ip1 - ydiff_i * g_i);
  }
  if (sys_size == 1) {
    c[1] = g[0] / diag[0];
  } else {
    /* LDL^T of the symmetric tridiagonal system (linalg/tridiag.c). */
    const int N = sys_size;
    double *gamma = (double *)malloc(sizeof(double) * (size_t)N);
    double *alpha = (double *)malloc(sizeof(double) * (size_t)N);
    double *cc = (double *)malloc(sizeof(double) * (size_t)N);
    double *z = (double *)malloc(sizeof(double) * (size_t)N);
    alpha[0] = diag[0];
    gamma[0] = offdiag[0] / alpha[0];
    for (int i = 1; i < N - 1; i++) {
      alpha[i] = diag[i] - offdiag[i - 1] * gamma[i - 1];
      gamma[i] = offdiag[i] / alpha[i];
    }
    if (N > 1) alpha[N - 1] = diag[N - 1] - offdiag[N - 2] * gamma[N - 2];
    z[0] = g[0];
    for (int i = 1; i < N; i++) z[i] = g[i] - gamma[i - 1] * z[i - 1];
    for (int i = 0; i < N; i++) cc[i] = z[i] / alpha[i];
    double *xs = c + 1;
    xs[N - 1] = cc[N - 1];
    if (N >= 2) {
      for (int i = N - 2, j = 0; j <= N - 2; j++, i--) xs[i] = cc[i] - gamma[i] * xs[i + 1];
    }
    free(gamma); free(alpha); free(cc); free(z);
  }
  /* gsl_interp_bsearch over [0, size-1] */
  int ilo = 0, ihi = size - 1;
  while (ihi > ilo + 1) {
    int i = (ihi + ilo) / 2;
    if (xa[i] > x) ihi = i; else ilo = i;
  }
  double y;
  const double x_hi = xa[ilo + 1], x_lo = xa[ilo];
  const double dx = x_hi - x_lo;
  if (dx > 0.0) {
    const double y_lo = ya[ilo], y_hi = ya[ilo + 1];
    const double dy = y_hi - y_lo;
    const double delx = x - x_lo;
    const double c_i = c[ilo], c_ip1 = c[ilo + 1];
    const double b_i = (dy / dx) - dx * (c_ip1 + 2.0 * c_i) / 3.0;
    const double d_i = (c_ip1 - c_i) / (3.0 * dx);
    y = y_lo + delx * (b_i + delx * (c_i + delx * d_i));
  } else {
    y = NAN;
  }
  free(c); free(g); free(diag); free(offdiag);
  return y;
}

/* ------------------------------------------------------------------------- */
/* Atmosphere: readATMpar (.cc:24-71), readnhFromFile (.cc:73-147),          */
/* MakeAtmosphere (.cc:920-942), FillInAirRefractiveIndex (.cc:193-213).      */
/* ------------------------------------------------------------------------- */
int or_parse_atmosphere(const char *text, size_t len, double pi, or_medium *m) {
  memset(m, 0, sizeof(*m));
  m->pi = pi;
  m->A_air = 1.00;
  m->A_ice = 1.78; m->B_ice = -0.43; m->C_ice = 0.0132;
  m->A_const = 1.00;

  /* readATMpar */
  {
    or_stream s = {text, text + len, 0};
    int n1 = 0;
    double d[5] = {0, 0, 0, 0, 0};
    while (st_getline(&s)) {
      if (n1 < 4)
        for (int i = 0; i < 5; i++) st_read_double(&s, &d[i]);
      if (n1 == 0) for (int i = 0; i < 5; i++) m->atmlay[i] = d[i];
      if (n1 == 1) for (int i = 0; i < 5; i++) m->abc[i][0] = d[i];
      if (n1 == 2) for (int i = 0; i < 5; i++) m->abc[i][1] = d[i];
      if (n1 == 3) for (int i = 0; i < 5; i++) m->abc[i][2] = d[i];
      n1++;
    }
    for (int k = 0; k < 3; k++) m->abc[4][k] = m->abc[3][k];
    m->atmlay[4] = 150000 * 100;
  }

  /* readnhFromFile: collect groups exactly as the push/clear logic does. */
  size_t cap = len / 8 + 16;
  double *h = (double *)malloc(sizeof(double) * cap);
  double *nv = (double *)malloc(sizeof(double) * cap);
  int ngroups = 0;
  int group_end[16];
  size_t npts = 0;
  {
    or_stream s = {text, text + len, 0};
    for (int i = 0; i < 5; i++) st_ignore(&s, 256, '\n');
    int layer = 0;
    double d1 = 0, d2 = 0;
    while (st_getline(&s)) {
      st_read_double(&s, &d1);
      st_read_double(&s, &d2);
      if (d1 > -1) {
        if (npts >= cap) { cap *= 2; h = realloc(h, sizeof(double) * cap); nv = realloc(nv, sizeof(double) * cap); }
        h[npts] = d1; nv[npts] = d2; npts++;
        if (d1 * 100 >= m->atmlay[layer]) {
          if (layer > 0) { if (ngroups < 16) group_end[ngroups] = (int)npts; ngroups++; }
          layer++;
          if (layer > 4) layer = 4; /* ATMLAY has 5 entries; 1.5e7 cm is never reached */
        }
      }
    }
    if (layer > 0) { if (ngroups < 16) group_end[ngroups] = (int)npts; ngroups++; }
  }
  /* GSL's cspline needs >= 3 knots (gsl_spline_alloc fails, and the reference's default GSL
   * error handler aborts, .cc:932); a profile past the ATMLAY bounds (more than 4 air layers)
   * makes the reference index ATMLAY out of range (.cc:110).  Both are rejected, as the library
   * rejects them (airice_host.cpp). */
  if (ngroups < 1 || ngroups + 1 > 4 || npts < 4) { free(h); free(nv); return -1; }
  /* drop the duplicated last data point from the last group (.cc:138-140) */
  npts -= 1;
  group_end[ngroups - 1] -= 1;
  m->max_layers = ngroups + 1;
  m->n_points = (int)npts;
  m->h_top = h[npts - 1];
  for (int i = 0; i < ngroups && i < 8; i++)
    m->layer_sizes[i] = group_end[i] - (i ? group_end[i - 1] : 0);

  /* spline over the flattened profile; only n(0) is ever used (.cc:203) */
  const double N0s = or_spline_eval_at(h, nv, (int)npts, 0.0);
  free(h); free(nv);

  double N0 = 0;
  for (int il = 0; il < 5; il++) {
    double hlow = m->atmlay[il] / 100;
    m->C_air[il] = 1.0 / (m->abc[il][2] / 100);
    if (il > 0) N0 = m->A_air + m->B_air[il - 1] * exp(-hlow * m->C_air[il - 1]);
    if (il == 0) { N0 = N0s; m->N0 = N0s; }
    m->B_air[il] = ((N0 - 1) / exp(-hlow * m->C_air[il]));
  }
  return 0;
}

int or_load_atmosphere(const char *path, double pi, or_medium *m) {
  FILE *f = fopen(path, "rb");
  if (!f) return -1;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char *buf = (char *)malloc((size_t)n + 1);
  size_t got = fread(buf, 1, (size_t)n, f);
  fclose(f);
  buf[got] = 0;
  int rc = or_parse_atmosphere(buf, got, pi, m);
  free(buf);
  return rc;
}

/* ------------------------------------------------------------------------- */
/* Medium model (.cc:150-191, 216-263)                                        */
/* ------------------------------------------------------------------------- */
static double GetB_ice(const or_medium *m, double z) { (void)z; return m->B_ice; }
static double GetC_ice(const or_medium *m, double z) { (void)z; return m->C_ice; }
double or_getnz_ice(const or_medium *m, double z) {
  z = fabs(z);
  return m->A_ice + GetB_ice(m, z) * exp(-GetC_ice(m, z) * z);
}

static int air_layer(const or_medium *m, double z) {
  double zabs = fabs(z);
  int which = 0;
  for (int il = 0; il < m->max_layers - 1; il++) {
    if (zabs < m->atmlay[il + 1] / 100 && zabs >= m->atmlay[il] / 100) { which = il; il = 100; }
  }
  if (zabs >= m->atmlay[m->max_layers - 1] / 100) which = m->max_layers - 1;
  return which;
}
/* pythonwrapper AirIceRayTracing.cc:173-238 (UseConstantRefractiveIndex branches) */
static double GetB_air(const or_medium *m, double z) {
  return m->constant_air_index ? 0 : m->B_air[air_layer(m, z)];
}
static double GetC_air(const or_medium *m, double z) {
  return m->constant_air_index ? 1e-9 : m->C_air[air_layer(m, z)];
}
double or_getnz_air(const or_medium *m, double z) {
  double zabs = fabs(z);
  if (m->constant_air_index) return m->A_const;
  return m->A_air + GetB_air(m, zabs) * exp(-GetC_air(m, zabs) * zabs);
}

/* Fresnel amplitude transmission (.cc:285-337) */
static double Trans_S(const or_medium *m, double thetai, double ice_h) {
  double n1 = or_getnz_air(m, ice_h), n2 = or_getnz_ice(m, 0);
  double a = (n1 / n2) * (sin(thetai));
  double sqterm = sqrt(1 - a * a);
  double num = n1 * cos(thetai) - n2 * sqterm;
  double den = n1 * cos(thetai) + n2 * sqterm;
  double tS = 1 + (num / den);
  if (isnan(tS)) tS = 0;
  return tS;
}
static double Trans_P(const or_medium *m, double thetai, double ice_h) {
  double n1 = or_getnz_air(m, ice_h), n2 = or_getnz_ice(m, 0);
  double a = (n1 / n2) * (sin(thetai));
  double sqterm = sqrt(1 - a * a);
  double num = n1 * sqterm - n2 * cos(thetai);
  double den = n1 * sqterm + n2 * cos(thetai);
  double tP = (1 - (num / den)) * (n1 / n2);
  if (isnan(tP)) tP = 0;
  return tP;
}

/* ------------------------------------------------------------------------- */
/* Analytic antiderivatives (.cc:377-447)                                     */
/* ------------------------------------------------------------------------- */
static double fDnfR(double x, double A, double B, double C, double L) {
  double y = A + B * exp(C * x);
  return (L / C) * (1.0 / sqrt(A * A - L * L)) *
         (C * x - log(A * (A + B * exp(C * x)) - L * L + sqrt(A * A - L * L) * sqrt(y * y - L * L)));
}

static double ftimeD(const or_medium *m, double x, double A, double C, double Speedc, double L,
                     int air_or_ice) {
  double n = air_or_ice ? or_getnz_air(m, x) : or_getnz_ice(m, x);
  double n2 = n * n; /* pow(Getnz(x),2) */
  return (1.0 / (Speedc * C * sqrt(n2 - L * L))) *
         (n2 - L * L +
          (C * x - log(A * n - L * L + sqrt(A * A - L * L) * sqrt(n2 - L * L))) *
              (A * A * sqrt(n2 - L * L)) / sqrt(A * A - L * L) +
          A * sqrt(n2 - L * L) * log(n + sqrt(n2 - L * L)));
}

static double fpathD(double x, double A, double B, double C, double L) {
  double e = exp(C * x);
  double e2 = exp(2 * C * x);
  double y = A + B * e;
  double Q = (A * A + 2 * A * B * e + B * B * e2 - L * L) / (y * y);
  double sA = sqrt(A * A - L * L);
  return (log(y * (sqrt(Q) + 1)) -
          (A * log(A * sA * sqrt(Q) + B * sA * e * sqrt(Q) + A * A + A * B * e - L * L)) / sA +
          (A * C * x) / sA) / C;
}

/* GetRayHorizontalPath / PropagationTime / GeometricPath (.cc:449-513) */
static double GetRayHorizontalPath(const or_medium *m, double A, double Rx, double Tx, double L, int air) {
  double Ba, Ca, Bb, Cb;
  if (air) { Ba = GetB_air(m, Rx); Ca = -GetC_air(m, Rx); Bb = GetB_air(m, Tx); Cb = -GetC_air(m, Tx); }
  else     { Ba = GetB_ice(m, Rx); Ca = -GetC_ice(m, Rx); Bb = GetB_ice(m, Tx); Cb = -GetC_ice(m, Tx); }
  double x1 = +fDnfR(Rx, A, Ba, Ca, L) - fDnfR(Tx, A, Bb, Cb, L);
  if (air) x1 *= -1;
  return x1;
}
static double GetRayPropagationTime(const or_medium *m, double A, double Rx, double Tx, double L, int air) {
  double Ca, Cb;
  if (air) { Ca = -GetC_air(m, Rx); Cb = -GetC_air(m, Tx); }
  else     { Ca = -GetC_ice(m, Rx); Cb = -GetC_ice(m, Tx); }
  double t = +ftimeD(m, Rx, A, Ca, SPEEDC, L, air) - ftimeD(m, Tx, A, Cb, SPEEDC, L, air);
  if (air) t *= -1;
  return t;
}
static double GetRayGeometricPath(const or_medium *m, double A, double Rx, double Tx, double L, int air) {
  double Ba, Ca, Bb, Cb;
  if (air) { Ba = GetB_air(m, Rx); Ca = -GetC_air(m, Rx); Bb = GetB_air(m, Tx); Cb = -GetC_air(m, Tx); }
  else     { Ba = GetB_ice(m, Rx); Ca = -GetC_ice(m, Rx); Bb = GetB_ice(m, Tx); Cb = -GetC_ice(m, Tx); }
  double g = fpathD(Rx, A, Ba, Ca, L) - fpathD(Tx, A, Bb, Cb, L);
  if (air) g *= -1;
  return g;
}

/* GetLayerHitPointPar (.cc:521-646): {THD, Recv deg, L, t, geo} */
void or_layer_hit_point_par(const or_medium *m, double n_layer1, double Rx, double Tx,
                            double IncidentAng, int air, double out[5]) {
  const double pi = m->pi;
  double SurfaceRayIncidentAngle = IncidentAng * (pi / 180.0);
  double A, nzRx, nzTx;
  if (air) { A = m->A_air; nzRx = or_getnz_air(m, Rx); nzTx = or_getnz_air(m, Tx); }
  else     { A = m->A_ice; nzRx = or_getnz_ice(m, Rx); nzTx = or_getnz_ice(m, Tx); }
  double RayAngleInside2ndLayer = asin((n_layer1 / nzTx) * sin(SurfaceRayIncidentAngle));
  double Lang = RayAngleInside2ndLayer;
  double ReceiveAngle;
  if (air) ReceiveAngle = asin((or_getnz_air(m, Tx) * sin(Lang)) / or_getnz_air(m, Rx));
  else     ReceiveAngle = asin((or_getnz_ice(m, Tx) * sin(Lang)) / or_getnz_ice(m, Rx));
  double Lvalue = nzRx * sin(ReceiveAngle);
  out[0] = GetRayHorizontalPath(m, A, Rx, Tx, Lvalue, air);
  out[1] = ReceiveAngle * (180 / pi);
  out[2] = Lvalue;
  out[3] = GetRayPropagationTime(m, A, Rx, Tx, Lvalue, air);
  out[4] = GetRayGeometricPath(m, A, Rx, Tx, Lvalue, air);
}

/* Layer skip scans (.cc:1798-1825 == .cc:666-690). */
static int skip_above(const or_medium *m, double txh) {
  int skip = 0;
  for (int il = m->max_layers; il > -1; il--) {
    /* ATMLAY[il-1] is read only when the first test holds (txh < ATMLAY[0]/100 = 0 at il=0) */
    if (txh < m->atmlay[il] / 100 && (il - 1 >= 0 ? txh >= m->atmlay[il - 1] / 100 : 0)) il = -100;
    if (il > -1) skip++;
  }
  return skip;
}
static int skip_below(const or_medium *m, double ice_h) {
  int skip = 0;
  for (int il = 0; il < m->max_layers; il++) {
    if (ice_h >= m->atmlay[il] / 100 && ice_h < m->atmlay[il + 1] / 100) il = 100;
    if (il < m->max_layers) skip++;
  }
  return skip;
}

/* GetRayTracingSolutions (.cc:1796-2017) */
void or_ray_solution(const or_medium *m, double RayLaunchAngleInAir, double AirTxHeight,
                     double IceLayerHeight, double AntennaDepth, int InIce, double dummy[18]) {
  const double pi = m->pi;
  int SkipLayersAbove = skip_above(m, AirTxHeight);
  int SkipLayersBelow = skip_below(m, IceLayerHeight);
  double Start_nh = 0, StartHeight = 0, StopHeight = 0, StartAngle = 0;
  double THDair = 0, GeoAir = 0, TimeAir = 0;
  const int top = m->max_layers - SkipLayersAbove - 1;
  for (int il = top; il > SkipLayersBelow - 1; il--) {
    if (il == top) StartHeight = AirTxHeight;
    else StartHeight = m->atmlay[il + 1] / 100 - 0.00001;
    Start_nh = or_getnz_air(m, StartHeight);
    if (il == (SkipLayersBelow - 1) + 1) StopHeight = IceLayerHeight;
    else StopHeight = m->atmlay[il] / 100;
    if (il == top) StartAngle = 180 - RayLaunchAngleInAir;
    double hp[5];
    or_layer_hit_point_par(m, Start_nh, StopHeight, StartHeight, StartAngle, 1, hp);
    THDair += hp[0];
    StartAngle = hp[1];
    TimeAir += hp[3];
    GeoAir += hp[4];
  }
  double IncidentAngleonIce = StartAngle;
  double THDice = 0, GeoIce = 0, TimeIce = 0, RecvIce = 0;
  if (InIce) {
    /* TransitionBoundary==0 branch (.cc:1897-1922) */
    double StartDepth = 0.0;
    Start_nh = or_getnz_air(m, IceLayerHeight);
    double StopDepth = -AntennaDepth;
    StartAngle = IncidentAngleonIce;
    double hp[5];
    or_layer_hit_point_par(m, Start_nh, StopDepth, StartDepth, StartAngle, 0, hp);
    THDice += hp[0];
    StartAngle = hp[1];
    TimeIce += hp[3];
    GeoIce += hp[4];
    RecvIce = hp[1];
  }
  for (int i = 0; i < 18; i++) dummy[i] = 0;
  dummy[0] = 0;
  dummy[1] = AirTxHeight;
  dummy[2] = THDair + THDice;
  dummy[3] = THDair;
  dummy[4] = THDice;
  dummy[5] = (TimeIce + TimeAir) * SPEEDC;
  dummy[6] = TimeAir * SPEEDC;
  dummy[7] = TimeIce * SPEEDC;
  dummy[8] = (TimeIce + TimeAir) * 1e9;
  dummy[9] = TimeAir * 1e9;
  dummy[10] = TimeIce * 1e9;
  dummy[11] = RayLaunchAngleInAir;
  dummy[12] = IncidentAngleonIce;
  dummy[13] = RecvIce;
  dummy[14] = Trans_S(m, IncidentAngleonIce * (pi / 180.0), IceLayerHeight);
  dummy[15] = Trans_P(m, IncidentAngleonIce * (pi / 180.0), IceLayerHeight);
  dummy[16] = GeoAir;
  dummy[17] = GeoIce;
}

/* MakeRayTracingTable grid arithmetic (.cc:12-21, 2019-2061). */
void or_grid_init(or_grid *g, double depth_cm, double ice_cm, double height_step,
                  double start_angle, double stop_angle, double angle_step) {
  g->in_ice = depth_cm < 0;
  g->depth_m = depth_cm / 100;
  g->ice_m = ice_cm / 100;
  g->start_height = 100000;
  g->stop_height = g->in_ice ? g->ice_m : g->ice_m + g->depth_m;
  g->height_step = height_step;
  g->height_steps = (int)floor((g->start_height - g->stop_height) / height_step) + 1;
  g->start_angle = start_angle;
  g->stop_angle = stop_angle;
  g->angle_step = angle_step;
  g->angle_steps = (int)floor((stop_angle - start_angle) / angle_step) + 1;
  /* .cc:2081-2082: rows whose unforced AirTxHeight is not > 0 push nothing, and heights fall
     with the row index, so the table holds the leading rows only */
  g->table_rows = g->height_steps;
  while (g->table_rows > 0 && !(g->start_height - g->height_step * (g->table_rows - 1) > 0))
    g->table_rows--;
}

/* Table columns (.cc:2101-2111): dummy indices */
static const int TABLE_COL[11] = {1, 2, 7, 6, 11, 3, 14, 15, 16, 17, 13};

void or_table_rows(const or_medium *m, const or_grid *g, int row0, int row1, float *table,
                   double *full, size_t ld, int nthreads) {
  const int na = g->angle_steps;
  const long total = (long)(row1 - row0) * na;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 64) if (nthreads > 0)
#endif
  for (long k = 0; k < total; k++) {
    int ihei = row0 + (int)(k / na);
    int iang = (int)(k % na);
    double H = g->start_height - g->height_step * ihei;
    if (!(H > 0)) continue; /* .cc:2082 */
    double th = g->start_angle + g->angle_step * iang;
    if (H != g->stop_height && ihei == g->height_steps - 1) H = g->stop_height;
    if (iang == na - 1) th = g->stop_angle;
    double d[18];
    or_ray_solution(m, th, H, g->stop_height, g->depth_m, g->in_ice, d);
    size_t r = (size_t)(ihei - row0) * na + iang;
    if (table) for (int c = 0; c < 11; c++) table[c * ld + r] = (float)d[TABLE_COL[c]];
    if (full) for (int c = 0; c < 18; c++) full[c * ld + r] = d[c];
  }
}

/* ------------------------------------------------------------------------- */
/* Minimizer path                                                             */
/* ------------------------------------------------------------------------- */
/* GetAirPropagationPar (.cc:661-804): out[5*ML+2]; returns filled layers. */
static int air_propagation(const or_medium *m, double LaunchAngleAir, double AirTxHeight,
                           double IceLayerHeight, double *out) {
  const double pi = m->pi;
  int SkipLayersAbove = skip_above(m, AirTxHeight);
  int SkipLayersBelow = skip_below(m, IceLayerHeight);
  double StartAngle = 0, StartHeight = 0, Start_nh = 0, StopHeight = 0;
  double L0 = 0;
  int nf = 0;
  const int top = m->max_layers - SkipLayersAbove - 1;
  for (int il = top; il > SkipLayersBelow - 1; il--) {
    if (il == top) StartHeight = AirTxHeight;
    else StartHeight = m->atmlay[il + 1] / 100 - 0.00001;
    Start_nh = or_getnz_air(m, StartHeight);
    if (il == (SkipLayersBelow - 1) + 1) StopHeight = IceLayerHeight;
    else StopHeight = m->atmlay[il] / 100;
    if (il == top) StartAngle = 180 - LaunchAngleAir;
    if (il == top) {
      double hp[5];
      or_layer_hit_point_par(m, Start_nh, StopHeight, StartHeight, StartAngle, 1, hp);
      for (int j = 0; j < 5; j++) out[nf * 5 + j] = hp[j];
      L0 = hp[2];
      StartAngle = hp[1];
      nf++;
    }
    if (il < top) {
      double nzStop = or_getnz_air(m, StopHeight);
      double RecAng = asin(L0 / nzStop);
      RecAng = RecAng * (180 / pi);
      out[nf * 5 + 0] = GetRayHorizontalPath(m, m->A_air, StopHeight, StartHeight, L0, 1);
      out[nf * 5 + 1] = RecAng;
      out[nf * 5 + 2] = L0;
      out[nf * 5 + 3] = GetRayPropagationTime(m, m->A_air, StopHeight, StartHeight, L0, 1);
      out[nf * 5 + 4] = GetRayGeometricPath(m, m->A_air, StopHeight, StartHeight, L0, 1);
      StartAngle = RecAng;
      nf++;
    }
  }
  out[5 * m->max_layers + 1] = nf;
  return nf;
}

/* GetIcePropagationPar (.cc:807-869), TransitionBoundary==0 branch. */
static void ice_propagation(const or_medium *m, double IceLayerHeight, double AntennaDepth,
                            double Lvalue, double out[5]) {
  (void)IceLayerHeight;
  const double pi = m->pi;
  double StartDepth = 0.0, StopDepth = AntennaDepth;
  double nzStopDepth = or_getnz_ice(m, StopDepth);
  out[0] = GetRayHorizontalPath(m, m->A_ice, StopDepth, StartDepth, Lvalue, 0);
  out[1] = asin(Lvalue / nzStopDepth) * (180 / pi);
  out[2] = Lvalue;
  out[3] = GetRayPropagationTime(m, m->A_ice, StopDepth, StartDepth, Lvalue, 0);
  out[4] = GetRayGeometricPath(m, m->A_ice, StopDepth, StartDepth, Lvalue, 0);
}

typedef struct { double airtxheight, icelayerheight, antennadepth, horizontaldistance; } minp;

/* MinimizeforLaunchAngle (.cc:873-917) */
static double MinimizeforLaunchAngle(const or_medium *m, double x, const minp *p) {
  double out[5 * 8 + 2];
  int nf = air_propagation(m, x, p->airtxheight, p->icelayerheight, out);
  double thd_air = 0;
  for (int i = 0; i < nf; i++) thd_air += out[i * 5];
  /* nf==0 (Tx above 150 km or below the ice): the reference reads out[-4] and an
   * unset out[2] (UB); modelled as NaN. */
  double L = nf > 0 ? out[2] : NAN;
  double thd_ice = 0;
  if (p->antennadepth != 0) {
    double ic[5];
    ice_propagation(m, p->icelayerheight, p->antennadepth, L, ic);
    thd_ice += ic[0];
  }
  return (p->horizontaldistance - (thd_ice + thd_air));
}

/* RayTracingFunctions:: scalar layer (RayTracingFunctions.cc): the same formulas as the
 * MultiRay restatements above in the RTF layouts -- GetLayerHitPointPar (.cc:399-527) and
 * GetIcePropagationPar (.cc:661-681) 4-wide {THD, Recv deg, L, t}, GetAirPropagationPar
 * (.cc:529-659) 4 x MaxLayers + count at [4*MaxLayers], GetRayOpticalPath (.cc:349-369),
 * GetRayPropagationTime (.cc:371-397), fDnfR (.cc:293-303), ftimeD (.cc:328-347),
 * MinimizeforLaunchAngle (.cc:683-731).  Op codes as AIRICE_RTF_* (include/airice.h). */
int or_rtf_eval(const or_medium *m, int op, const double *a, double *out) {
  double t[5 * 8 + 2];
  switch (op) {
    case 0: /* HIT_POINT */
      or_layer_hit_point_par(m, a[0], a[1], a[2], a[3], (int)a[4], t);
      for (int j = 0; j < 4; j++) out[j] = t[j];
      return 4;
    case 1: /* OPTICAL_PATH */
      out[0] = GetRayHorizontalPath(m, a[0], a[1], a[2], a[3], (int)a[4]);
      return 1;
    case 2: /* PROPAGATION_TIME */
      out[0] = GetRayPropagationTime(m, a[0], a[1], a[2], a[3], (int)a[4]);
      return 1;
    case 3: { /* AIR_PROPAGATION */
      for (int j = 0; j < 5 * 8 + 2; j++) t[j] = 0;
      int nf = air_propagation(m, a[0], a[1], a[2], t);
      for (int j = 0; j < 4 * m->max_layers + 1; j++) out[j] = 0;
      for (int i = 0; i < nf; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = t[5 * i + j];
      out[4 * m->max_layers] = nf;
      return 4 * m->max_layers + 1;
    }
    case 4: /* ICE_PROPAGATION (IncidentAngleonIce unused, .cc:664) */
      ice_propagation(m, a[1], a[2], a[3], t);
      for (int j = 0; j < 4; j++) out[j] = t[j];
      return 4;
    case 5: /* FDNFR */
      out[0] = fDnfR(a[0], a[1], a[2], a[3], a[4]);
      return 1;
    case 6: /* FTIMED (b unused by the formula) */
      out[0] = ftimeD(m, a[0], a[1], a[3], a[4], a[5], (int)a[6]);
      return 1;
    case 7: { /* MIN_LAUNCH */
      minp p = {a[1], a[2], a[3], a[4]};
      out[0] = MinimizeforLaunchAngle(m, a[0], &p);
      return 1;
    }
    case 8: /* AIR2ICE: the Air2IceRayTracing CLI solve */
      or_rtf_air2ice(m, a[0], a[1], a[2], a[3], out);
      return 16;
    /* MultiRayAirIceRefraction:: forms (AIRICE_MR_*): the restatements above, 5-wide */
    case 9: /* MR_FPATHD (x, a, b, c, speedc, l) */
      out[0] = fpathD(a[0], a[1], a[2], a[3], a[5]);
      return 1;
    case 10: /* MR_GEOMETRIC_PATH */
      out[0] = GetRayGeometricPath(m, a[0], a[1], a[2], a[3], (int)a[4]);
      return 1;
    case 11: /* MR_HIT_POINT */
      or_layer_hit_point_par(m, a[0], a[1], a[2], a[3], (int)a[4], out);
      return 5;
    case 12: { /* MR_AIR_PROPAGATION */
      for (int j = 0; j < 5 * m->max_layers + 2; j++) out[j] = 0;
      air_propagation(m, a[0], a[1], a[2], out);
      return 5 * m->max_layers + 2;
    }
    case 13: /* MR_ICE_PROPAGATION */
      ice_propagation(m, a[1], a[2], a[3], out);
      return 5;
    case 14: { /* MR_MIN_LAUNCH */
      minp p = {a[1], a[2], a[3], a[4]};
      out[0] = MinimizeforLaunchAngle(m, a[0], &p);
      return 1;
    }
    default:
      return -1;
  }
}

/* FindFunctionRoot (.cc:340-374) with GSL bisection semantics:
 * gsl_root_fsolver_set (fsolver.c) + bisection_init/bisection_iterate (bisection.c) +
 * gsl_root_test_interval(lo, hi, 0, tol) (convergence.c), loop while CONTINUE and
 * iter < max_iter, return the last root.  Uninitialised-state cases (a non-finite
 * endpoint) are modelled as a zero-filled state. */
double or_bisect(or_fn f, void *ctx, double x_lo, double x_hi, double tol, int max_iter,
                 int *status) {
  double root, lo, hi, f_lower = 0.0, f_upper = 0.0;
  if (x_lo > x_hi) { *status |= OR_SOLVE_BAD_BRACKET; return 0.0; }
  root = 0.5 * (x_lo + x_hi);
  lo = x_lo; hi = x_hi;
  {
    double fl = f(lo, ctx);
    if (!isfinite(fl)) { *status |= OR_SOLVE_NONFINITE_END; goto loop; }
    double fu = f(hi, ctx);
    if (!isfinite(fu)) { *status |= OR_SOLVE_NONFINITE_END; goto loop; }
    f_lower = fl; f_upper = fu;
  }
loop:;
  int iter = 0;
  int cont;
  double r = 0;
  do {
    iter++;
    /* bisection_iterate */
    if (f_lower == 0.0) { root = lo; hi = lo; }
    else if (f_upper == 0.0) { root = hi; lo = hi; }
    else {
      double xb = (lo + hi) / 2.0;
      double fb = f(xb, ctx);
      if (!isfinite(fb)) {
        *status |= OR_SOLVE_STALE_MID; /* EBADFUNC: no state change */
      } else if (fb == 0.0) {
        root = xb; lo = xb; hi = xb;
      } else if ((f_lower > 0.0 && fb < 0.0) || (f_lower < 0.0 && fb > 0.0)) {
        root = 0.5 * (lo + xb); hi = xb; f_upper = fb;
      } else {
        root = 0.5 * (xb + hi); lo = xb; f_lower = fb;
      }
    }
    r = root;
    /* gsl_root_test_interval(lo, hi, 0, tol) */
    if (lo > hi) { cont = 0; }
    else {
      double min_abs = ((lo > 0.0 && hi > 0.0) || (lo < 0.0 && hi < 0.0))
                           ? (fabs(lo) < fabs(hi) ? fabs(lo) : fabs(hi)) : 0;
      double tolerance = 0 + tol * min_abs;
      cont = !(fabs(hi - lo) < tolerance);
    }
  } while (cont && iter < max_iter);
  if (cont) *status |= OR_SOLVE_MAXITER;
  return r;
}

typedef struct { const or_medium *m; const minp *p; } minctx;
static double min_cb(double x, void *c) {
  const minctx *mc = (const minctx *)c;
  return MinimizeforLaunchAngle(mc->m, x, mc->p);
}
static double bisection_root(const or_medium *m, const minp *p, double x_lo, double x_hi,
                             double tol, int max_iter, int *status) {
  minctx c = {m, p};
  return or_bisect(min_cb, &c, x_lo, x_hi, tol, max_iter, status);
}

/* gsl_root_fsolver_brent (GNU GSL 2.x roots/brent.c, brent_init / brent_iterate; GSL is absent
 * from this image: restated from its published algorithm, parity unpinned by reference output)
 * under RayTracingFunctions::FindFunctionRoot (RayTracingFunctions.cc:256-290: max_iter 20,
 * gsl_root_test_interval(lo, hi, 0, tol)).  Uninitialised-state cases as in or_bisect: a
 * non-finite f at a bracket end leaves a zero state (flag NONFINITE_END); a non-finite f at an
 * iterate stores nothing (STALE_MID); lower > upper fails set (BAD_BRACKET, root 0). */
double or_brent(or_fn f, void *ctx, double x_lo, double x_hi, double tol_rel, int max_iter,
                int *status, int *iters) {
  const double EPS = 2.2204460492503131e-16; /* GSL_DBL_EPSILON */
  if (x_lo > x_hi) { *status |= OR_SOLVE_BAD_BRACKET; *iters = 0; return 0.0; }
  double root = 0.5 * (x_lo + x_hi), lo = x_lo, hi = x_hi;
  double a = 0, b = 0, c = 0, d = 0, e = 0, fa = 0, fb = 0, fc = 0;
  double fl = f(x_lo, ctx), fu = 0;
  int ok = isfinite(fl);
  if (ok) { fu = f(x_hi, ctx); ok = isfinite(fu); }
  if (!ok) *status |= OR_SOLVE_NONFINITE_END;
  else {
    a = x_lo; fa = fl; b = x_hi; fb = fu; c = x_hi; fc = fu;
    d = x_hi - x_lo; e = x_hi - x_lo;
  }
  int iter = 0, cont;
  do {
    iter++;
    double la = a, lb = b, lc = c, ld = d, le = e, lfa = fa, lfb = fb, lfc = fc;
    int ac_equal = 0;
    if ((lfb < 0 && lfc < 0) || (lfb > 0 && lfc > 0)) {
      ac_equal = 1; lc = la; lfc = lfa; ld = lb - la; le = lb - la;
    }
    if (fabs(lfc) < fabs(lfb)) {
      ac_equal = 1; la = lb; lb = lc; lc = la; lfa = lfb; lfb = lfc; lfc = lfa;
    }
    double tol = 0.5 * EPS * fabs(lb);
    double mm = 0.5 * (lc - lb);
    if (lfb == 0) { root = lb; lo = lb; hi = lb; }
    else if (fabs(mm) <= tol) {
      root = lb;
      if (lb < lc) { lo = lb; hi = lc; } else { lo = lc; hi = lb; }
    } else {
      if (fabs(le) < tol || fabs(lfa) <= fabs(lfb)) { ld = mm; le = mm; }
      else {
        double p, q, r, sr = lfb / lfa;
        if (ac_equal) { p = 2 * mm * sr; q = 1 - sr; }
        else {
          q = lfa / lfc; r = lfb / lfc;
          p = sr * (2 * mm * q * (q - r) - (lb - la) * (r - 1));
          q = (q - 1) * (r - 1) * (sr - 1);
        }
        if (p > 0) q = -q; else p = -p;
        double t1 = 3 * mm * q - fabs(tol * q), t2 = fabs(le * q);
        if (2 * p < (t1 < t2 ? t1 : t2)) { le = ld; ld = p / q; }
        else { ld = mm; le = mm; }
      }
      la = lb; lfa = lfb;
      if (fabs(ld) > tol) lb += ld; else lb += (mm > 0 ? +tol : -tol);
      double fnew = f(lb, ctx);
      if (!isfinite(fnew)) *status |= OR_SOLVE_STALE_MID;
      else {
        lfb = fnew;
        a = la; b = lb; c = lc; d = ld; e = le; fa = lfa; fb = lfb; fc = lfc;
        root = lb;
        double cc = lc;
        if ((lfb < 0 && lfc < 0) || (lfb > 0 && lfc > 0)) cc = la;
        if (lb < cc) { lo = lb; hi = cc; } else { lo = cc; hi = lb; }
      }
    }
    if (lo > hi) cont = 0;
    else {
      double min_abs = ((lo > 0.0 && hi > 0.0) || (lo < 0.0 && hi < 0.0))
                           ? (fabs(lo) < fabs(hi) ? fabs(lo) : fabs(hi)) : 0;
      cont = !(fabs(hi - lo) < 0 + tol_rel * min_abs);
    }
  } while (cont && iter < max_iter);
  if (cont) *status |= OR_SOLVE_MAXITER;
  *iters = iter;
  return root;
}

/* Air2IceRayTracing CLI solve (Air2IceRayTracing.C:56-185) on the RayTracingFunctions layer:
 * straight-line angle, bracket [thR-16, thR] with the 0.05-degree probe (90.00 threshold), Brent,
 * then GetAirPropagationPar / GetIcePropagationPar at the root.  out[16]: include/airice.h
 * AIRICE_RTF_AIR2ICE_FIELDS. */
void or_rtf_air2ice(const or_medium *m, double AirTxHeight, double HorizontalDistance,
                    double IceLayerHeight, double AntennaDepth, double *o) {
  const double pi = m->pi;
  double StraightAngle = 180 - (atan(HorizontalDistance / (AirTxHeight - IceLayerHeight + AntennaDepth)) * (180.0 / pi));
  double startanglelim = StraightAngle - 16, endanglelim = StraightAngle;
  int probes = 0;
  double out[5 * 8 + 2];
  if (startanglelim < 90.00) {
    startanglelim = 90.05;
    int checknan = 0;
    while (checknan == 0 && startanglelim > 89.9) {
      int nf = air_propagation(m, startanglelim, AirTxHeight, IceLayerHeight, out);
      double t = 0;
      for (int i = 0; i < nf; i++) t += out[i * 5];
      if ((isnan(t) == 0 && t > 0) || startanglelim > endanglelim - 1) checknan = 1;
      else { startanglelim = startanglelim + 0.05; probes++; }
    }
  }
  if (endanglelim < 90.001 && endanglelim > 90.00) endanglelim = 90.05;
  minp p = {AirTxHeight, IceLayerHeight, AntennaDepth, HorizontalDistance};
  minctx c = {m, &p};
  int status = 0, iters = 0;
  double LaunchAngleAir = or_brent(min_cb, &c, startanglelim, endanglelim, 0.000000001, 20,
                                   &status, &iters);
  int nf = air_propagation(m, LaunchAngleAir, AirTxHeight, IceLayerHeight, out);
  double thd_air = 0, t_air = 0;
  for (int i = 0; i < nf; i++) { thd_air += out[i * 5]; t_air += out[3 + i * 5] * pow(10, 9); }
  double L = nf > 0 ? out[2] : NAN;
  double inc = nf > 0 ? out[1 + (nf - 1) * 5] : NAN;
  double ic[5];
  ice_propagation(m, IceLayerHeight, AntennaDepth, L, ic);
  double t_ice = ic[3] * pow(10, 9);
  o[0] = startanglelim; o[1] = endanglelim; o[2] = LaunchAngleAir; o[3] = thd_air;
  o[4] = inc; o[5] = L; o[6] = t_air; o[7] = ic[0]; o[8] = ic[1]; o[9] = t_ice;
  o[10] = ic[0] + thd_air; o[11] = t_ice + t_air;
  o[12] = status | (nf == 0 ? OR_SOLVE_NO_AIR_LAYER : 0); o[13] = iters; o[14] = probes; o[15] = nf;
}

double or_straight_angle(const or_medium *m, double H, double D, double ice, double depth) {
  double thR = 0;
  if (depth < 0) thR = 180 - (atan(D / (H - ice - depth)) * (180.0 / m->pi));
  if (depth >= 0) thR = 180 - (atan(D / (H - (ice + depth))) * (180.0 / m->pi));
  return thR;
}

/* Bracket set-up shared by both variants (.cc:1472-1516, AirIceRayTracing.cc:937-987). */
static double bracket_and_solve(const or_medium *m, double AirTxHeight, double HorizontalDistance,
                                double *IceLayerHeight, double *AntennaDepth, double StraightAngle,
                                minp *p, int *status) {
  if (*AntennaDepth >= 0) {
    *IceLayerHeight = *AntennaDepth + *IceLayerHeight;
    *AntennaDepth = 0;
    p->airtxheight = AirTxHeight; p->icelayerheight = *IceLayerHeight;
    p->antennadepth = *AntennaDepth; p->horizontaldistance = HorizontalDistance;
  }
  if (*AntennaDepth < 0) {
    p->airtxheight = AirTxHeight; p->icelayerheight = *IceLayerHeight;
    p->antennadepth = -*AntennaDepth; p->horizontaldistance = HorizontalDistance;
  }
  double lo = StraightAngle - 16;
  double hi = StraightAngle;
  if (m->constant_air_index) {
    lo = 90; /* pythonwrapper AirIceRayTracing.cc:978-980 */
  } else if (lo < 90.001) {
    lo = 90.001;
    int checknan = 0;
    double out[5 * 8 + 2];
    while (checknan == 0 && lo > 89.9) {
      int nf = air_propagation(m, lo, AirTxHeight, *IceLayerHeight, out);
      double s = 0;
      for (int i = 0; i < nf; i++) s += out[i * 5];
      if ((isnan(s) == 0 && s > 0) || lo > hi - 0.1) checknan = 1;
      else { lo = lo + 0.05; *status |= OR_SOLVE_PROBED; }
    }
  }
  if (hi < 90.001 && hi > 90.00) hi = 90.05;
  return bisection_root(m, p, lo, hi, 0.000000001, 40, status);
}

/* Air2IceRayTracing (.cc:1464-1616) */
int or_air2ice(const or_medium *m, double AirTxHeight, double HorizontalDistance,
               double IceLayerHeight, double AntennaDepth, double StraightAngle, double dummy[17]) {
  const double pi = m->pi;
  int status = 0;
  minp p;
  double LaunchAngleAir = bracket_and_solve(m, AirTxHeight, HorizontalDistance, &IceLayerHeight,
                                            &AntennaDepth, StraightAngle, &p, &status);
  double out[5 * 8 + 2];
  int nf = air_propagation(m, LaunchAngleAir, AirTxHeight, IceLayerHeight, out);
  double thd_air = 0, t_air = 0, geo_air = 0;
  for (int i = 0; i < nf; i++) { thd_air += out[i * 5]; t_air += out[3 + i * 5]; geo_air += out[4 + i * 5]; }
  double L = nf > 0 ? out[2] : NAN;
  double inc = nf > 0 ? out[1 + (nf - 1) * 5] : NAN;
  if (nf == 0) status |= OR_SOLVE_NO_AIR_LAYER;
  double thd_ice = 0, ant = 0, t_ice = 0, geo_ice = 0;
  if (AntennaDepth < 0) {
    double ic[5];
    ice_propagation(m, IceLayerHeight, -AntennaDepth, L, ic);
    thd_ice = ic[0]; ant = ic[1]; t_ice = ic[3]; geo_ice = ic[4];
  }
  double thd = thd_ice + thd_air;
  double tt = t_ice + t_air;
  dummy[0] = AirTxHeight;
  dummy[1] = thd;
  dummy[2] = thd_air;
  dummy[3] = thd_ice;
  dummy[4] = tt * SPEEDC;
  dummy[5] = t_ice * SPEEDC;
  dummy[6] = t_air * SPEEDC;
  dummy[7] = tt;
  dummy[8] = t_ice;
  dummy[9] = t_air;
  dummy[10] = LaunchAngleAir;
  dummy[11] = ant;
  dummy[12] = Trans_S(m, inc * (pi / 180.0), IceLayerHeight);
  dummy[13] = Trans_P(m, inc * (pi / 180.0), IceLayerHeight);
  dummy[14] = geo_air;
  dummy[15] = geo_ice;
  dummy[16] = inc;
  return status;
}

void or_solve_batch(const or_medium *m, const double *txh, const double *dist, const double *depth,
                    double ice_h, size_t n, double *out, size_t ld, uint8_t *status, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16) if (nthreads > 0)
#endif
  for (long i = 0; i < (long)n; i++) {
    double thR = or_straight_angle(m, txh[i], dist[i], ice_h, depth[i]);
    double d[17];
    int st = or_air2ice(m, txh[i], dist[i], ice_h, depth[i], thR, d);
    for (int c = 0; c < 17; c++) out[c * ld + i] = d[c];
    if (status) status[i] = (uint8_t)st;
  }
}

/* GetHorizontalDistanceToIntersectionPoint (.cc:945-989) */
int or_hdtip(const or_medium *m, double Src, double Dist, double Depth, double Ice, double o[9]) {
  const double pi = m->pi;
  double H = Src / 100, D = Dist / 100, I = Ice / 100, d = Depth / 100;
  double thR = or_straight_angle(m, H, D, I, d);
  double dm[17];
  or_air2ice(m, H, D, I, d, thR, dm);
  o[0] = dm[5] * 100;   /* opticalPathLengthInIce */
  o[1] = dm[6] * 100;   /* opticalPathLengthInAir */
  o[2] = dm[15] * 100;  /* geometricalPathLengthInIce */
  o[3] = dm[14] * 100;  /* geometricalPathLengthInAir */
  o[4] = dm[10] * (pi / 180);
  o[5] = dm[2] * 100;
  o[6] = dm[12];
  o[7] = dm[13];
  o[8] = dm[11] * (pi / 180);
  int ok = 0;
  if ((fabs(dm[1] - D) / D < 0.01 && D <= 100) || (fabs(dm[1] - D) < 1 && D > 100)) ok = 1;
  if (dm[1] < 0) ok = 0;
  return ok;
}

/* or_hdtip over a batch (cm), OpenMP: out 9 columns (stride ld), ok[i] the returned bool,
 * status[i] the Air2IceRayTracing status bits of the solve behind it (masks the reference-UB rows) */
void or_hdtip_batch(const or_medium *m, const double *src_cm, const double *dist_cm,
                    const double *depth_cm, double ice_cm, size_t n, double *out, size_t ld,
                    uint8_t *ok, uint8_t *status, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16) if (nthreads > 0)
#endif
  for (long i = 0; i < (long)n; i++) {
    double o[9];
    ok[i] = (uint8_t)or_hdtip(m, src_cm[i], dist_cm[i], depth_cm[i], ice_cm, o);
    for (int c = 0; c < 9; c++) out[c * ld + i] = o[c];
    if (status) {
      const double H = src_cm[i] / 100, D = dist_cm[i] / 100, I = ice_cm / 100, d = depth_cm[i] / 100;
      double dm[17];
      status[i] = (uint8_t)or_air2ice(m, H, D, I, d, or_straight_angle(m, H, D, I, d), dm);
    }
  }
}

/* ------------------------------------------------------------------------- */
/* pythonwrapper variant (pythonwrapper/AirIceRayTracing.cc, TraceIceToAir.C) */
/* ------------------------------------------------------------------------- */
int or_py_air2ice(const or_medium *m, double AirTxHeight, double HorizontalDistance,
                  double IceLayerHeight, double AntennaDepth, double StraightAngle, double dummy[15]) {
  const double pi = m->pi;
  int status = 0;
  minp p;
  double LaunchAngleAir = bracket_and_solve(m, AirTxHeight, HorizontalDistance, &IceLayerHeight,
                                            &AntennaDepth, StraightAngle, &p, &status);
  double out[5 * 8 + 2];
  int nf = air_propagation(m, LaunchAngleAir, AirTxHeight, IceLayerHeight, out);
  double thd_air = 0, t_air = 0, geo_air = 0;
  for (int i = 0; i < nf; i++) { thd_air += out[i * 5]; t_air += out[3 + i * 5]; geo_air += out[4 + i * 5]; }
  double L = nf > 0 ? out[2] : NAN;
  double inc = nf > 0 ? out[1 + (nf - 1) * 5] : NAN;
  if (nf == 0) status |= OR_SOLVE_NO_AIR_LAYER;
  double thd_ice = 0, ant = 0, t_ice = 0, geo_ice = 0;
  if (AntennaDepth < 0) {
    double ic[5];
    ice_propagation(m, IceLayerHeight, -AntennaDepth, L, ic);
    thd_ice = ic[0]; ant = ic[1]; t_ice = ic[3]; geo_ice = ic[4];
  }
  double thd = thd_ice + thd_air;
  double tt = t_ice + t_air;
  dummy[0] = AirTxHeight;
  dummy[1] = thd;
  dummy[2] = thd_air;
  dummy[3] = thd_ice;
  dummy[4] = tt * SPEEDC;
  dummy[5] = t_ice * SPEEDC;
  dummy[6] = t_air * SPEEDC;
  dummy[7] = tt;
  dummy[8] = t_ice;
  dummy[9] = t_air;
  dummy[10] = LaunchAngleAir;
  dummy[11] = asin((or_getnz_air(m, IceLayerHeight) / or_getnz_ice(m, 0)) * sin(inc * (pi / 180))) * (180. / pi);
  dummy[12] = ant;
  dummy[13] = geo_air;
  dummy[14] = geo_ice;
  return status;
}

int or_py_trace_ice_to_air(const or_medium *m, double AntennaDepth, double IceLayerHeight,
                           double AirTxHeight, double HorizontalDistance, double a[10]) {
  /* GetRayTracingSolution (AirIceRayTracing.cc:884-927), metres */
  double thR = or_straight_angle(m, AirTxHeight, HorizontalDistance, IceLayerHeight, AntennaDepth);
  double dm[15];
  int st = or_py_air2ice(m, AirTxHeight, HorizontalDistance, IceLayerHeight, AntennaDepth, thR, dm);
  double geo_ice = dm[14], geo_air = dm[13];
  double launch = dm[10], hd = dm[2], aoi = dm[11], recv = dm[12];
  int ok = 0;
  if ((fabs(dm[1] - HorizontalDistance) / HorizontalDistance < 0.01 && HorizontalDistance <= 100) ||
      (fabs(dm[1] - HorizontalDistance) < 1 && HorizontalDistance > 100))
    ok = 1;
  if (dm[1] < 0) ok = 0;
  /* TraceIceToAir.C:33-34: swap(launch, recv); recv = 180 - recv */
  double t = launch; launch = recv; recv = t;
  recv = 180 - recv;
  if (ok) {
    a[0] = AirTxHeight; a[1] = HorizontalDistance; a[2] = geo_ice; a[3] = geo_air;
    a[4] = launch; a[5] = recv; a[6] = hd; a[7] = aoi; a[8] = 0; a[9] = 0;
  } else {
    for (int i = 0; i < 10; i++) a[i] = -1000;
  }
  (void)st;
  return ok;
}

void or_py_trace_batch(const or_medium *m, const double *depth, const double *ice,
                       const double *txh, const double *dist, size_t n, double *out10, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16) if (nthreads > 0)
#endif
  for (long i = 0; i < (long)n; i++)
    or_py_trace_ice_to_air(m, depth[i], ice[i], txh[i], dist[i], out10 + 10 * i);
}

/* ------------------------------------------------------------------------- */
/* Table lookup (.cc:992-1462)                                                */
/* ------------------------------------------------------------------------- */
static double lk_interp(double x, double xa, double ya, double xb, double yb) {
  return ya + (yb - ya) * ((x - xa) / (xb - xa)); /* .cc:992-995 */
}

/* bounded column read; out of range -> NaN and the UB flag (the reference reads past the vector) */
static double lk_at(const or_lookup_table *t, int c, long i, int *flags) {
  if (i < 0 || i >= t->n) { *flags |= OR_LK_UNPINNED; return NAN; }
  return (double)t->col[c][i];
}

/* FindClosestAirTxHeight (.cc:1033-1126) */
static void lk_closest_txh(const or_lookup_table *t, double P, long *s1, long *e1, double *c1,
                           long *s2, long *e2, double *c2, int *flags) {
  int CurrentHeightStep = (int)floor((P - t->LoopStopHeight) / t->HeightStepSize);
  int Index = t->TotalHeightSteps - CurrentHeightStep - 1;
  long MaxAngleBin = (long)Index * t->TotalAngleSteps + t->TotalAngleSteps - 1;
  long MinAngleBin = (long)Index * t->TotalAngleSteps + 0;
  double val = -0.001;
  long StartBin = MaxAngleBin;
  int went = 0;
  while ((val != 0 && val < 0.01) || isnan(val)) {
    if (StartBin < 0) { *flags |= OR_LK_UNPINNED; break; }
    val = lk_at(t, 1, StartBin, flags);
    StartBin--;
    went = 1;
  }
  if (went) StartBin = StartBin + 1;
  val = -0.001;
  long EndBin = MinAngleBin;
  went = 0;
  while ((val != 0 && val < 0.01) || isnan(val)) {
    if (EndBin >= t->n) { *flags |= OR_LK_UNPINNED; break; }
    val = lk_at(t, 1, EndBin, flags);
    EndBin++;
    went = 1;
  }
  if (went) EndBin = EndBin - 1;
  *s1 = EndBin;
  *e1 = StartBin;
  *c1 = fabs(lk_at(t, 0, Index, flags) - P); /* sic: row index used as a ray index */
  *s2 = *s1 - t->TotalAngleSteps;
  *e2 = *e1 - t->TotalAngleSteps;
  if (*s2 < 0) *s2 = *s1 + t->TotalAngleSteps;
  if (*e2 < 0) *e2 = *e1 + t->TotalAngleSteps;
  *c2 = fabs(lk_at(t, 0, Index, flags) - P);
}

/* FindClosestTHD (.cc:1128-1169) */
static void lk_closest_thd(const or_lookup_table *t, double P, long StartIndex, long EndIndex,
                           long *rs, long *re, double *cv, int *flags) {
  long MidIndex;
  for (int i = 0; i < 8; i++) {
    if (EndIndex - StartIndex >= 3) {
      MidIndex = (long)floor((double)((StartIndex + EndIndex) / 2));
      if (lk_at(t, 1, MidIndex, flags) - P > 0) StartIndex = MidIndex;
      if (lk_at(t, 1, MidIndex, flags) - P < 0) EndIndex = MidIndex;
    }
  }
  double minimum = 100000000000;
  long index2 = 0;
  for (long ipnt = StartIndex; ipnt < EndIndex + 1; ipnt++) {
    double v = lk_at(t, 1, ipnt, flags);
    double minval = fabs(v - P);
    if (minval < minimum && v > P) {
      minimum = minval;
    } else {
      index2 = ipnt;
      break;
    }
  }
  long index1 = index2 - 1;
  minimum = fabs(P - lk_at(t, 1, index2, flags));
  if (minimum > fabs(P - lk_at(t, 1, index1, flags))) minimum = fabs(P - lk_at(t, 1, index1, flags));
  *rs = index1;
  *re = index2;
  *cv = minimum;
}

/* GetParValues (.cc:1172-1302) */
static void lk_par_values(const or_lookup_table *t, double H, double D, double *H1, double Par1[10],
                          double *H2, double Par2[10], int *flags) {
  long TotalTableEntries = t->n - 1;
  double MinAirTxHeight = lk_at(t, 0, TotalTableEntries, flags);
  long si[4] = {0, 0, 0, 0}, ei[4] = {0, 0, 0, 0};
  double cv[3] = {0, 0, 0};
  lk_closest_txh(t, H, &si[0], &ei[0], &cv[0], &si[2], &ei[2], &cv[2], flags);
  *H1 = lk_at(t, 0, si[0], flags);
  double MaxTHD = lk_at(t, 1, si[0], flags);
  if (D <= MaxTHD) {
    lk_closest_thd(t, D, si[0], ei[0], &si[1], &ei[1], &cv[1], flags);
    if (cv[1] != 0) {
      double x1 = lk_at(t, 1, si[1], flags), x2 = lk_at(t, 1, ei[1], flags);
      for (int ip = 0; ip < 10; ip++)
        Par1[ip] = lk_interp(D, x1, lk_at(t, 1 + ip, si[1], flags), x2, lk_at(t, 1 + ip, ei[1], flags));
    }
    if (cv[1] == 0) {
      si[1] = si[1] + 1;
      ei[1] = si[1];
      for (int ip = 0; ip < 10; ip++) Par1[ip] = lk_at(t, 1 + ip, si[1], flags);
    }
  } else {
    for (int ip = 0; ip < 10; ip++) Par1[ip] = -1e9;
  }
  if (cv[0] != 0 && H > MinAirTxHeight && si[2] < TotalTableEntries) {
    *H2 = lk_at(t, 0, si[2], flags);
    MaxTHD = lk_at(t, 1, si[2], flags);
    if (D <= MaxTHD) {
      lk_closest_thd(t, D, si[2], ei[2], &si[3], &ei[3], &cv[2], flags);
      if (cv[2] != 0) {
        double x1 = lk_at(t, 1, si[3], flags), x2 = lk_at(t, 1, ei[3], flags);
        for (int ip = 0; ip < 10; ip++)
          Par2[ip] = lk_interp(D, x1, lk_at(t, 1 + ip, si[3], flags), x2, lk_at(t, 1 + ip, ei[3], flags));
      }
      if (cv[2] == 0) {
        si[3] = si[3] + 1;
        ei[3] = si[3];
        for (int ip = 0; ip < 10; ip++) Par2[ip] = lk_at(t, 1 + ip, si[3], flags);
      }
    } else {
      for (int ip = 0; ip < 10; ip++) Par2[ip] = -1e9;
    }
  } else {
    *H2 = *H1;
    for (int ip = 0; ip < 10; ip++) Par2[ip] = Par1[ip];
  }
}

/* The table walks above, exported for the tests of the C++ drop-in's FindClosestAirTxHeight /
 * FindClosestTHD / GetParValues (test infrastructure, like everything here). */
void or_lookup_closest_txh(const or_lookup_table *t, double P, long out_idx[4], double out_c[2],
                           int *flags) {
  lk_closest_txh(t, P, &out_idx[0], &out_idx[1], &out_c[0], &out_idx[2], &out_idx[3], &out_c[1],
                 flags);
}
void or_lookup_closest_thd(const or_lookup_table *t, double P, long s, long e, long out_idx[2],
                           double *c, int *flags) {
  lk_closest_thd(t, P, s, e, &out_idx[0], &out_idx[1], c, flags);
}
void or_lookup_par_values(const or_lookup_table *t, double H, double D, double out[22],
                          int *flags) {
  lk_par_values(t, H, D, &out[0], out + 1, &out[11], out + 12, flags);
}

/* GetHorizontalDistanceToIntersectionPoint_Table (.cc:1305-1462); AntennaNumber already
 * resolved to the table `t`.  Slots the reference leaves uninitialised are returned as 0
 * with OR_LK_UNPINNED set. */
int or_table_lookup(const or_medium *m, const or_lookup_table *t, double SrcHeightASL,
                    double HorizontalDistanceToRx, double RxDepthBelowIceBoundary,
                    double IceLayerHeight, double o[9], int *flags) {
  const double pi = m->pi;
  *flags = 0;
  double AirTxHeight = SrcHeightASL / 100;
  double HorizontalDistance = HorizontalDistanceToRx / 100;
  IceLayerHeight = IceLayerHeight / 100;
  int CheckSolution = 1;
  long TotalTableEntries = t->n - 1;
  double MaxAirTxHeight = lk_at(t, 0, 0, flags);
  double MinAirTxHeight = lk_at(t, 0, TotalTableEntries, flags);
  double x1 = 0, x2 = 0, y1 = 0, y2 = 0;
  double Par1[15], Par2[15], piv[15];
  int set[15];
  for (int i = 0; i < 15; i++) { piv[i] = 0; set[i] = 0; }
  if (AirTxHeight <= MaxAirTxHeight && AirTxHeight >= MinAirTxHeight && AirTxHeight > 0) {
    double H1, H2;
    lk_par_values(t, AirTxHeight, HorizontalDistance, &H1, Par1, &H2, Par2, flags);
    x1 = H1;
    x2 = H2;
    for (int ipar = 0; ipar < 10; ipar++) {
      y1 = Par1[ipar];
      y2 = Par2[ipar];
      double v = 0;
      int checkval = (y1 == -1e9 || y2 == -1e9);
      if (x1 != x2 && checkval == 0) {
        v = lk_interp(AirTxHeight, x1, y1, x2, y2);
      } else {
        if (x1 == x2 && y1 == y2) v = Par1[ipar];
        if (y2 == -1e9 && y1 == -1e9) ipar = 9;
      }
      piv[ipar] = v;
      set[ipar] = 1;
    }
  }
  for (int i = 0; i < 10; i++)
    if (!set[i]) *flags |= OR_LK_UNPINNED;
  double THD = piv[0];
  o[0] = piv[1] * 100; /* opticalPathLengthInIce */
  o[1] = piv[2] * 100; /* opticalPathLengthInAir */
  o[2] = piv[8] * 100; /* geometricalPathLengthInIce */
  o[3] = piv[7] * 100; /* geometricalPathLengthInAir */
  o[4] = piv[3] * (pi / 180);
  o[5] = piv[4] * 100;
  o[6] = piv[5];
  o[7] = piv[6];
  o[8] = piv[9] * (pi / 180);
  int CheckSolBool = 0;
  int one = (y1 == -1e9 && y2 != -1e9) || (y2 == -1e9 && y1 != -1e9);
  if (one) {
    /* .cc:1419: cm arguments scaled by 100 again, optical/geometric slots swapped */
    double f[9];
    CheckSolBool = or_hdtip(m, SrcHeightASL * 100, HorizontalDistanceToRx * 100,
                            RxDepthBelowIceBoundary * 100, IceLayerHeight * 100, f);
    o[2] = f[0]; o[3] = f[1]; o[0] = f[2]; o[1] = f[3];
    o[4] = f[4]; o[5] = f[5]; o[6] = f[6]; o[7] = f[7]; o[8] = f[8];
    *flags |= OR_LK_FALLBACK;
  }
  if (y2 == -1e9 && y1 == -1e9) CheckSolution = 0;
  if (one && CheckSolBool == 0) CheckSolution = 0;
  if (AirTxHeight > MaxAirTxHeight) CheckSolution = 0;
  if (AirTxHeight < MinAirTxHeight) CheckSolution = 0;
  if (AirTxHeight < 0) CheckSolution = 0;
  if (o[4] < 0) CheckSolution = 0;
  if ((fabs(THD - HorizontalDistance) / HorizontalDistance > 0.01 && HorizontalDistance <= 100) ||
      (fabs(THD - HorizontalDistance) > 1 && HorizontalDistance > 100))
    CheckSolution = 0;
  if (CheckSolution == 0) { o[0] = 0; o[1] = 0; o[4] = 0; o[5] = 0; }
  return CheckSolution;
}

void or_table_lookup_batch(const or_medium *m, const or_lookup_table *t, const double *src_cm,
                           const double *dist_cm, const double *depth_cm, double ice_cm, size_t n,
                           double *out, size_t ld, unsigned char *ok, unsigned char *flags,
                           int nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#else
  (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 256) num_threads(nthreads)
  for (long i = 0; i < (long)n; ++i) {
    double o[9];
    int fl = 0;
    ok[i] = (unsigned char)or_table_lookup(m, t, src_cm[i], dist_cm[i], depth_cm[i], ice_cm, o, &fl);
    flags[i] = (unsigned char)fl;
    for (int c = 0; c < 9; ++c) out[(size_t)c * ld + (size_t)i] = o[c];
  }
}

/* ------------------------------------------------------------------------- */
/* SingleRayAirIceRefraction.C:33-299 (RayTracingFunctions.cc numerics)       */
/* ------------------------------------------------------------------------- */
int or_single_ray_trace(const or_medium *m, double AntennaDepth, double RayLaunchAngle,
                        double AirTxHeight, double IceLayerHeight, or_single_ray *out, double *xs,
                        double *zs, long cap) {
  const double pi = m->pi;
  memset(out, 0, sizeof(*out));
  const int ML = m->max_layers;
  const int SkipLayersAbove = skip_above(m, AirTxHeight);   /* :60-71 */
  const int SkipLayersBelow = skip_below(m, IceLayerHeight); /* :75-86 */
  out->skip_above = SkipLayersAbove;
  out->skip_below = SkipLayersBelow;
  /* air layer loop (:100-154) */
  double StartHeight = 0, StopHeight = 0, StartAngle = 0, TotalHorizontalDistance = 0, Lvalue = 0;
  for (int ilayer = ML - SkipLayersAbove - 1; ilayer > SkipLayersBelow - 1; ilayer--) {
    if (ilayer == ML - SkipLayersAbove - 1) StartHeight = AirTxHeight;
    else StartHeight = m->atmlay[ilayer + 1] / 100 - 0.00001;
    double Start_nh = or_getnz_air(m, StartHeight);
    if (ilayer == (SkipLayersBelow - 1) + 1) StopHeight = IceLayerHeight;
    else StopHeight = m->atmlay[ilayer] / 100;
    if (ilayer == ML - SkipLayersAbove - 1) {
      StartAngle = 180 - RayLaunchAngle;
      double hp[5];
      or_layer_hit_point_par(m, Start_nh, StopHeight, StartHeight, StartAngle, 1, hp);
      TotalHorizontalDistance += hp[0];
      StartAngle = hp[1];
      Lvalue = hp[2];
    } else {
      double nzStopHeight = or_getnz_air(m, StopHeight);
      double RecAng = asin(Lvalue / nzStopHeight);
      RecAng = RecAng * (180 / pi);
      double THD = GetRayHorizontalPath(m, m->A_air, StopHeight, StartHeight, Lvalue, 1);
      TotalHorizontalDistance += THD;
      StartAngle = RecAng;
    }
  }
  out->thd_air = TotalHorizontalDistance;
  out->inc_ice = StartAngle;
  out->L = Lvalue;
  /* GetIcePropagationPar (RayTracingFunctions.cc:661-679) with positive depth */
  {
    double nzStopDepth = or_getnz_ice(m, AntennaDepth);
    out->thd_ice = GetRayHorizontalPath(m, m->A_ice, AntennaDepth, 0.0, Lvalue, 0);
    out->recv_ice = asin(Lvalue / nzStopDepth) * (180 / pi);
    out->t_ice = GetRayPropagationTime(m, m->A_ice, AntennaDepth, 0.0, Lvalue, 0);
  }
  /* path sampler (:226-299) */
  const int nl = ML - SkipLayersAbove - SkipLayersBelow;
  out->n_layers = nl;
  long ip = 0;
  double LastRefracted_x = 0, LastHeight = 0, Refracted_x = 0;
  for (int il = 0; il < nl; il++) {
    double LayerStartHeight = (il == 0) ? AirTxHeight : LastHeight - 0.00001;
    double LayerStopHeight = (il == nl - 1) ? IceLayerHeight : (m->atmlay[nl - il - 1] / 100);
    for (double i = LayerStartHeight; i > LayerStopHeight - 1; i = i - 1) {
      if (i < LayerStopHeight) i = LayerStopHeight;
      double fa = fDnfR(-i, m->A_air, GetB_air(m, -i), GetC_air(m, -i), Lvalue);
      double fb = fDnfR(-(LayerStartHeight), m->A_air, GetB_air(m, -(LayerStartHeight)),
                        GetC_air(m, -(LayerStartHeight)), Lvalue);
      Refracted_x = fa - fb + LastRefracted_x;
      if (xs && ip < cap) { xs[ip] = Refracted_x; zs[ip] = i; }
      ip++;
      LastHeight = i;
    }
    LastRefracted_x = Refracted_x;
  }
  out->n_air = ip;
  for (int i = 0; i > -(AntennaDepth + 1); i--) {
    double fa = fDnfR((double)i, m->A_ice, GetB_ice(m, i), GetC_ice(m, i), Lvalue);
    double fb = fDnfR(0, m->A_ice, GetB_ice(m, 0), GetC_ice(m, 0), Lvalue);
    double refractedpath = LastRefracted_x - fa + fb;
    if (xs && ip < cap) { xs[ip] = refractedpath; zs[ip] = (double)i + IceLayerHeight; }
    ip++;
  }
  out->n_ice = ip - out->n_air;
  return 0;
}
