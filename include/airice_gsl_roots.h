/* airice_gsl_roots.h -- the two GNU GSL types in the reference's FindFunctionRoot signatures
 * (MultiRayAirIceRefraction.h:122, RayTracingFunctions.h:88, pythonwrapper/AirIceRayTracing.h:94):
 *
 *   double FindFunctionRoot(gsl_function F, double x_lo, double x_hi,
 *                           const gsl_root_fsolver_type *T, double tolerance [, int iterations]);
 *
 * A caller that has GNU GSL gets GSL's own declarations (and passes gsl_root_fsolver_bisection /
 * gsl_root_fsolver_brent from libgsl as usual).  Without GSL this header declares the same two types
 * with GSL's public layout (gsl/gsl_math.h: struct gsl_function_struct; gsl/gsl_roots.h: the
 * anonymous-struct typedef gsl_root_fsolver_type), so the functions keep the reference's mangled
 * names (e.g. _ZN16AirIceRayTracing16FindFunctionRootE19gsl_function_structddPK21gsl_root_fsolver_typedi),
 * and names the solver types this library provides under the GSL names by macro.
 *
 * The solver is selected by the type's name ("bisection", "brent"), so libgsl's own type objects
 * work too; the root search itself runs in libairice.so (GSL 2.x roots/bisection.c and
 * roots/brent.c semantics, compat_roots.cpp) on the caller's host function.  Other GSL solver types
 * abort with a message. */
#ifndef AIRICE_GSL_ROOTS_H
#define AIRICE_GSL_ROOTS_H

#include <stddef.h>

#if defined(__has_include)
#if __has_include(<gsl/gsl_roots.h>) && !defined(AIRICE_NO_SYSTEM_GSL)
#include <gsl/gsl_roots.h>
#define AIRICE_HAVE_GSL 1
#endif
#endif

#ifndef AIRICE_HAVE_GSL
#ifdef __cplusplus
extern "C" {
#endif
struct gsl_function_struct {
  double (*function)(double x, void *params);
  void *params;
};
typedef struct gsl_function_struct gsl_function;
typedef struct {
  const char *name;
  size_t size;
  int (*set)(void *state, gsl_function *f, double *root, double x_lower, double x_upper);
  int (*iterate)(void *state, gsl_function *f, double *root, double *x_lower, double *x_upper);
} gsl_root_fsolver_type;
/* this library's solver types (name "bisection" / "brent"); set/iterate are not callable */
extern const gsl_root_fsolver_type *const airice_root_fsolver_bisection;
extern const gsl_root_fsolver_type *const airice_root_fsolver_brent;
#ifdef __cplusplus
}
#endif
#define gsl_root_fsolver_bisection airice_root_fsolver_bisection
#define gsl_root_fsolver_brent airice_root_fsolver_brent
#endif

#endif /* AIRICE_GSL_ROOTS_H */
