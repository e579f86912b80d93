// airice_host.h -- host-only internals (airice_host.cpp): no HIP types, so the sanitizer harness
// (tests/cpp/asan_harness.cpp) builds them with a plain host compiler.
#pragma once
#include <string>

#include "airice.h"

namespace airice {

constexpr int kMaxParsedLayers = 4;  // ATMLAY has 5 bounds -> at most 4 air layers (.h:56)

// printf-style message for airice_last_error() (thread-local)
void set_error(const char* fmt, ...);
// pi of a reference namespace: MultiRayAirIceRefraction.h:29 / RayTracingFunctions.h:26
// (3.1415927) or pythonwrapper AirIceRayTracing.h:25 (4*atan(1))
double variant_pi(int variant);
// readATMpar + readnhFromFile + spline + FillInAirRefractiveIndex (.cc:24-213, 920-942) on a
// text image of a GDAS Atmosphere.dat, with the reference's stream semantics
int parse_gdas(const std::string& text, airice_medium* m);

}  // namespace airice
