// airice_internal.h -- host-side internals shared by the runtime and the launchers.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>

#include "airice.h"
#include "airice_device.hpp"
#include "airice_host.h"

namespace airice {

// Kernel-argument medium for one variant (pi) built from the parsed medium; the
// layer-boundary endpoints are evaluated here, on the host, once.
int build_dev_medium(const airice_medium* m, int variant, DevMedium* out);
// Batch-uniform ice endpoints: ice height ice_h (m) and antenna depth rx_depth (m, >= 0).
void build_ice_consts(const DevMedium& M, double ice_h, double rx_depth, IceConsts* out);

Endpoint host_air_endpoint(const DevMedium& M, double x);
Endpoint host_ice_endpoint(const DevMedium& M, double x);

int launch_table(const DevMedium& M, const IceConsts& I, const airice_grid* g, int row_begin,
                 int row_count, float* d_table, double* d_full, size_t ld, hipStream_t st);
int launch_table_multi(const DevMedium& M, const IceConsts* Ih, const airice_grid* grids, int n,
                       float* const* tables, const size_t* lds, hipStream_t st);
// entries of the table launch's per-grid caches (airice_table_cache_stats)
void table_cache_stats(int out[6]);
int launch_rays(const DevMedium& M, const IceConsts& I, const double* launch, const double* txh,
                int in_ice, size_t n, double* out, size_t ld, hipStream_t st);
void rays_host(const DevMedium& M, const IceConsts& I, const double* launch, const double* txh,
               int in_ice, size_t n, double* out, size_t ld);
// one query of the minimizer entry points on the host (airice_kernels.hip)
int solve_host_one(const DevMedium& M, const IceConsts& I, int variant, const double* in,
                   bool has_thr, double* out, uint8_t* status);
int hdtip_host_one(const DevMedium& M, const IceConsts& I, double ice_cm, const double* in,
                   double* out9, uint8_t* ok);
int trace_host_one(const DevMedium& M, const IceConsts& I, const double* in, double* out10);
int lookup_fallback_host_one(const DevMedium& M, const IceConsts& I, double ice_cm,
                             const double* in, double* out9, uint8_t* ok, const uint8_t* flags);
int launch_solve(const DevMedium& M, const IceConsts& I, int variant, const double* txh,
                 const double* dist, const double* depth, const double* thr, size_t n,
                 double* out, size_t ld, uint8_t* status, hipStream_t st);
int launch_hdtip(const DevMedium& M, const IceConsts& I, const double* src, const double* dist,
                 const double* depth, double ice_cm, size_t n, double* out, size_t ld,
                 uint8_t* ok, hipStream_t st);
// Stream-ordered scratch from a library-owned pool that keeps freed blocks (hipFreeAsync).
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t st);
// Batch size from which the minimizer groups the queries of source `in` batch-wide
// (AIRICE_GROUP_MIN overrides it; 0 when a source never groups by default).
size_t group_min_batch(int in);
// Table lookup: lookup_kernel, each AIRICE_LOOKUP_FALLBACK lane solving its minimizer fallback
// in place (airice_kernels.hip; the pack kernels: airice_lookup.hip).
int launch_lookup(const DevMedium& M, const IceConsts& I, const airice_lookup_table* t,
                  const double* src, const double* dist, const double* depth, double ice_cm,
                  size_t n, double* out, size_t ld, uint8_t* ok, uint8_t* flags, hipStream_t st);
int launch_lookup_pack(const airice_lookup_table* t, float* entries, hipStream_t st);
int launch_lookup_fallback(const DevMedium& M, const IceConsts& I, const double* src,
                           const double* dist, const double* depth, double ice_cm, size_t n,
                           double* out, size_t ld, uint8_t* ok, const uint8_t* flags,
                           hipStream_t st);
// SingleRayAirIceRefraction (airice_path.hip).  d_work: AIRICE_SINGLE_RAY_WORK doubles.
int plan_single_ray(const airice_medium* m, double depth, double launch, double txh, double ice,
                    airice_single_ray_info* info);
int launch_single_ray(const DevMedium& M, const airice_medium* m, double depth, double launch,
                      double txh, double ice, double* d_work, double* d_x, double* d_z,
                      size_t cap, hipStream_t st);
// RayTracingFunctions:: scalar layer (airice_rtf.hip): one call, one lane, d_out >= outputs
int rtf_outputs(int op, int max_layers);
int rtf_host(const DevMedium& M, int op, const double* args, size_t n_args, double* out);
// one-query calls on the host (airice_runtime.cpp): the mode, and per-thread cached folds
bool scalar_on_host();
int set_scalar_mode(int mode);
int folded_medium(const airice_medium* m, int variant, const DevMedium** out);
int folded_ice(const airice_medium* m, int variant, double ice_h, double rx_depth,
               const DevMedium** M, const IceConsts** I);
// one query of a minimizer entry point on the host, from an airice_medium (folds cached)
int solve_query_host(const airice_medium* m, int variant, double ice_h, const double* in,
                     bool has_thr, double* out, uint8_t* status);
int hdtip_query_host(const airice_medium* m, double ice_cm, const double* in, double* out9,
                     uint8_t* ok);
int trace_query_host(const airice_medium* m, const double* in, double* out10);
int launch_rtf(const DevMedium& M, int op, const double* args, size_t n_args, double* d_out,
               hipStream_t st);
int launch_trace(const DevMedium& M, const IceConsts& I, const double* depth, const double* ice,
                 const double* txh, const double* dist, size_t n, double* out10, hipStream_t st);

static_assert(kMaxParsedLayers == kMaxLayers, "parse and kernels agree on the layer count");

// One-query calls of the scalar drop-ins (the C++ MultiRayAirIceRefraction:: / RayTracingFunctions::
// functions, Py_TraceIceToAir, airice_rtf_eval): a pinned, device-mapped staging block per device
// that the host fills with the inputs and the kernels read and write in place (no copies), and a
// library-owned non-blocking stream; a call is its launches plus one wait.
// The slot of the current device (hipGetDevice) is created on first use and locked for the call.
// A call made of ONE kernel launch arms the slot's completion flag first (arm()); the launcher
// of that kernel takes the signal (take_scalar_signal) and passes it to the kernel, which stores
// the sequence number after its outputs (signal_done); sync() then spins on the pinned flag
// instead of synchronising the stream (launch + wait 7.8 us instead of 11-12 us).
struct ScalarSlot {
  double* h = nullptr;  // host view
  double* d = nullptr;  // device view of the same memory
  hipStream_t st = nullptr;
  unsigned* flag_h = nullptr;  // completion flag: host view
  unsigned* flag_d = nullptr;  //                  device view
  unsigned seq = 0;
};
constexpr size_t kScalarSlotDoubles = 512;
class ScalarCall {
 public:
  ScalarCall();  // on failure ok() is false and airice_last_error() says why
  ~ScalarCall();
  bool ok() const { return slot_ != nullptr; }
  ScalarSlot& slot() { return *slot_; }
  // Arms the completion signal for the next launch on this thread (the call's only kernel);
  // in[0 .. n_in-1] (n_in <= 4): the query inputs in the launcher's order, passed inline.
  void arm(const double* in = nullptr, int n_in = 0);
  // Waits for the call: on the flag when the armed signal was taken by a launcher (falling back
  // to the stream after a bounded spin), else on the slot's stream; AIRICE_OK or AIRICE_EHIP.
  int sync();
 private:
  ScalarSlot* slot_ = nullptr;
  void* lock_ = nullptr;
  bool armed_ = false;
};
// The armed signal of this thread (cleared by taking it); Signal{} when none is armed.
Signal take_scalar_signal();
// The table lookup's minimizer fallback for one query that lk_query flagged one-sided
// (.cc:1418-1420), on the device through the scalar slot: out9 / *ok as the batch lookup.
int lookup_fallback_one(const airice_medium* m, double src_cm, double dist_cm, double depth_cm,
                        double ice_cm, bool good, int flags, double out9[9], bool* ok);

// Kernel timing for the bench (airice_kernel_timing): when enabled, launches of the kernels
// below are bracketed by a hipEvent pair on their stream.  Off by default: one relaxed load.
enum KTimerId { KT_TABLE = 0, KT_ROOTS, KT_GROUP, KT_OUT, KT_LOOKUP, KT_COUNT };
extern std::atomic<bool> g_ktimer_on;
void ktimer_record(int id, bool begin, hipStream_t st);
inline void ktimer_begin(int id, hipStream_t st) {
  if (g_ktimer_on.load(std::memory_order_relaxed)) ktimer_record(id, true, st);
}
inline void ktimer_end(int id, hipStream_t st) {
  if (g_ktimer_on.load(std::memory_order_relaxed)) ktimer_record(id, false, st);
}

// Launch counters (airice_launch_count), always on: one relaxed increment per launch, so a test
// can assert that the kernel it means to check ran (a host route cannot pass for a device test).
enum LaunchId {
  LC_TABLE = 0,     // table_kernel (single- and multi-antenna)
  LC_RAYS,          // rays_kernel
  LC_SCALAR_RAY,    // scalar_ray_kernel (one-query GetRayTracingSolutions)
  LC_ROOTS,         // roots_kernel / roots_sorted_kernel (batched root finder)
  LC_SCALAR_SOLVE,  // scalar_solve_kernel (one-query minimizer entry points)
  LC_OUT,           // solve_out / hdtip_out / trace_out
  LC_LOOKUP,        // lookup_kernel
  LC_RTF,           // rtf_kernel (ray layer, GSL-Brent search)
  LC_SINGLE_RAY,    // single_ray_kernel
  LC_PATH,          // path_kernel
  LC_COUNT
};
extern std::atomic<long long> g_launches[LC_COUNT];
inline void count_launch(int id) { g_launches[id].fetch_add(1, std::memory_order_relaxed); }

}  // namespace airice
