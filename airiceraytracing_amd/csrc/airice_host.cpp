// airice_host.cpp -- the host-only part of libairice.so: error reporting, GDAS Atmosphere.dat
// ingestion and the MakeRayTracingTable grid set-up.  No HIP here, so the same file also builds
// into the sanitizer harness (tests/cpp/asan_harness.cpp, `make asan`).
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "airice.h"
#include "airice_host.h"

namespace airice {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

double variant_pi(int variant) {
  // MultiRayAirIceRefraction.h:29 / RayTracingFunctions.h:26 vs pythonwrapper AirIceRayTracing.h:25
  return variant == AIRICE_VARIANT_PYWRAPPER ? 4.0 * std::atan(1.0) : 3.1415927;
}

// Natural cubic spline through (xs, ys) evaluated at x: second-derivative system
// solved by symmetric-tridiagonal LDL^T, then the cubic on the bracketing interval
// (the algorithm of gsl_interp_cspline, which the reference uses for n(h=0) only).
static double natural_spline_at(const std::vector<double>& xs, const std::vector<double>& ys,
                                 double x) {
  const size_t n = xs.size();
  const size_t m = n - 2;  // interior unknowns
  std::vector<double> c(n, 0.0), rhs(m), dg(m), od(m);
  for (size_t i = 0; i < m; ++i) {
    const double h0 = xs[i + 1] - xs[i], h1 = xs[i + 2] - xs[i + 1];
    const double g0 = (h0 != 0.0) ? 1.0 / h0 : 0.0;
    const double g1 = (h1 != 0.0) ? 1.0 / h1 : 0.0;
    od[i] = h1;
    dg[i] = 2.0 * (h1 + h0);
    rhs[i] = 3.0 * ((ys[i + 2] - ys[i + 1]) * g1 - (ys[i + 1] - ys[i]) * g0);
  }
  if (m == 1) {
    c[1] = rhs[0] / dg[0];
  } else {
    std::vector<double> piv(m), lo(m), z(m);
    piv[0] = dg[0];
    lo[0] = od[0] / piv[0];
    for (size_t i = 1; i + 1 < m; ++i) {
      piv[i] = dg[i] - od[i - 1] * lo[i - 1];
      lo[i] = od[i] / piv[i];
    }
    piv[m - 1] = dg[m - 1] - od[m - 2] * lo[m - 2];
    z[0] = rhs[0];
    for (size_t i = 1; i < m; ++i) z[i] = rhs[i] - lo[i - 1] * z[i - 1];
    for (size_t i = 0; i < m; ++i) z[i] = z[i] / piv[i];
    c[m] = z[m - 1];
    for (size_t k = m - 1; k-- > 0;) c[k + 1] = z[k] - lo[k] * c[k + 2];
  }
  size_t a = 0, b = n - 1;
  while (b > a + 1) {
    const size_t mid = (a + b) / 2;
    if (xs[mid] > x) b = mid; else a = mid;
  }
  const double dx = xs[a + 1] - xs[a];
  if (!(dx > 0.0)) return NAN;
  const double dy = ys[a + 1] - ys[a];
  const double t = x - xs[a];
  const double bi = (dy / dx) - dx * (c[a + 1] + 2.0 * c[a]) / 3.0;
  const double di = (c[a + 1] - c[a]) / (3.0 * dx);
  return ys[a] + t * (bi + t * (c[a] + t * di));
}

// GDAS Atmosphere.dat ingestion with the reference's stream semantics
// (readATMpar .cc:24-71, readnhFromFile .cc:73-147, FillInAirRefractiveIndex .cc:193-213).
int parse_gdas(const std::string& text, airice_medium* m) {
  std::memset(m, 0, sizeof(*m));
  m->A_air = 1.00;
  m->A_ice = 1.78;
  m->B_ice = -0.43;
  m->C_ice = 0.0132;
  m->A_const = 1.00;
  {
    std::istringstream in(text);
    std::string line;
    int row = 0;
    double v[5] = {0, 0, 0, 0, 0};
    while (std::getline(in, line)) {
      if (row < 4) in >> v[0] >> v[1] >> v[2] >> v[3] >> v[4];
      if (row == 0) for (int i = 0; i < 5; ++i) m->atmlay_cm[i] = v[i];
      if (row >= 1 && row <= 3) for (int i = 0; i < 5; ++i) m->abc[i][row - 1] = v[i];
      ++row;
    }
    for (int k = 0; k < 3; ++k) m->abc[4][k] = m->abc[3][k];
    m->atmlay_cm[4] = 150000 * 100;
  }
  std::vector<double> hs, ns;
  int groups = 0;
  {
    std::istringstream in(text);
    for (int i = 0; i < 5; ++i) in.ignore(256, '\n');
    std::string line;
    int layer = 0;
    double h = 0, nv = 0;
    while (std::getline(in, line)) {
      in >> h >> nv;  // at EOF the last pair is seen twice (removed below, .cc:137-140)
      if (h > -1) {
        hs.push_back(h);
        ns.push_back(nv);
        if (h * 100 >= m->atmlay_cm[layer < 4 ? layer : 4]) {
          if (layer > 0) ++groups;
          ++layer;
        }
      }
    }
    if (layer > 0) ++groups;
  }
  if (groups < 1 || hs.size() < 4) {
    set_error("atmosphere: no refractive-index profile found");
    return AIRICE_EIO;
  }
  hs.pop_back();
  ns.pop_back();
  m->max_layers = groups + 1;
  m->n_points = (int32_t)hs.size();
  m->h_top = hs.back();
  if (m->max_layers > kMaxParsedLayers) {
    set_error("atmosphere: %d layers exceed the 5 ATMLAY bounds", m->max_layers);
    return AIRICE_EINVAL;
  }
  m->N0 = natural_spline_at(hs, ns, 0.0);
  double N0 = 0;
  for (int il = 0; il < 5; ++il) {
    const double hlow = m->atmlay_cm[il] / 100;
    m->C_air[il] = 1.0 / (m->abc[il][2] / 100);
    if (il > 0) N0 = m->A_air + m->B_air[il - 1] * std::exp(-hlow * m->C_air[il - 1]);
    if (il == 0) N0 = m->N0;
    m->B_air[il] = ((N0 - 1) / std::exp(-hlow * m->C_air[il]));
  }
  return AIRICE_OK;
}

// ---- table files (airice_table_save / _load) --------------------------------------------------
// The header is serialised field by field at fixed offsets (little-endian host), so that struct
// padding never reaches the file and the layout does not depend on the compiler.  The fields and
// columns are copied in host byte order, so the format is little-endian only because every host
// this library builds for is: a big-endian build is refused here rather than writing files whose
// magic and checksum would still match after a byte swap.
static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__,
              "table files are little-endian: host byte order is copied as is");
namespace {

constexpr char kTableMagic[8] = {'A', 'I', 'R', 'T', 'B', 'L', '0', '1'};
constexpr uint32_t kTableVersion = 1;

struct HeaderIO {
  unsigned char* buf;
  size_t off;
  bool store;
  template <class T>
  void f(T& v) {
    if (store) std::memcpy(buf + off, &v, sizeof(T));
    else std::memcpy(&v, buf + off, sizeof(T));
    off += sizeof(T);
  }
  void skip(size_t n) { off += n; }
};

void medium_io(HeaderIO& io, airice_medium& m) {
  for (double& v : m.atmlay_cm) io.f(v);
  for (auto& row : m.abc)
    for (double& v : row) io.f(v);
  for (double& v : m.B_air) io.f(v);
  for (double& v : m.C_air) io.f(v);
  io.f(m.N0);
  io.f(m.max_layers);
  io.f(m.n_points);
  io.f(m.A_air);
  io.f(m.A_ice);
  io.f(m.B_ice);
  io.f(m.C_ice);
  io.f(m.pi);
  io.f(m.h_top);
  io.f(m.constant_air_index);
  io.skip(4);
  io.f(m.A_const);
}

void grid_io(HeaderIO& io, airice_grid& g) {
  io.f(g.start_height);
  io.f(g.stop_height);
  io.f(g.height_step);
  io.f(g.height_steps);
  io.skip(4);
  io.f(g.start_angle);
  io.f(g.stop_angle);
  io.f(g.angle_step);
  io.f(g.angle_steps);
  io.skip(4);
  io.f(g.depth_m);
  io.f(g.ice_m);
  io.f(g.in_ice);
  io.f(g.table_rows);
}

// the parsed fields of two media, bit for bit (the variant's pi included)
bool same_medium(const airice_medium& a, const airice_medium& b) {
  unsigned char x[AIRICE_TABLE_FILE_HEADER] = {}, y[AIRICE_TABLE_FILE_HEADER] = {};
  airice_medium ca = a, cb = b;
  HeaderIO ia{x, 0, true}, ib{y, 0, true};
  medium_io(ia, ca);
  medium_io(ib, cb);
  return std::memcmp(x, y, ia.off) == 0;
}

inline uint64_t rotl64(uint64_t v, int r) { return (v << r) | (v >> (64 - r)); }

// four independent multiply-rotate lanes over 8-byte words (a non-cryptographic integrity check:
// catches truncation, bit rot and a file mixed up with another table)
uint64_t bytes_hash(const unsigned char* p, size_t n, uint64_t seed) {
  constexpr uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full;
  uint64_t h[4] = {seed ^ P1, seed ^ P2, seed + P1, seed - P2};
  size_t i = 0;
  for (; i + 32 <= n; i += 32) {
    for (int k = 0; k < 4; ++k) {
      uint64_t w;
      std::memcpy(&w, p + i + 8 * k, 8);
      h[k] = rotl64(h[k] + w * P2, 31) * P1;
    }
  }
  unsigned char tail[32] = {};
  std::memcpy(tail, p + i, n - i);
  for (int k = 0; k < 4; ++k) {
    uint64_t w;
    std::memcpy(&w, tail + 8 * k, 8);
    h[k] = rotl64(h[k] + w * P2, 31) * P1;
  }
  uint64_t r = rotl64(h[0], 1) + rotl64(h[1], 7) + rotl64(h[2], 12) + rotl64(h[3], 18) + n;
  r ^= r >> 33;
  r *= P2;
  r ^= r >> 29;
  return r;
}

struct FileCloser {
  FILE* f;
  ~FileCloser() {
    if (f) std::fclose(f);
  }
};

}  // namespace

}  // namespace airice

using namespace airice;

extern "C" {

const char* airice_last_error(void) { return g_err; }
const char* airice_version(void) { return "airice-mi355x 0.2.0 (gfx950, fp64; lookup pack format 2)"; }

int airice_atmosphere_parse(const char* text, size_t len, int variant, airice_medium* out) {
  if (text == nullptr || out == nullptr) {
    set_error("null argument");
    return AIRICE_EINVAL;
  }
  int rc = parse_gdas(std::string(text, len), out);
  if (rc == AIRICE_OK) out->pi = variant_pi(variant);
  return rc;
}

int airice_atmosphere_load(const char* path, int variant, airice_medium* out) {
  if (path == nullptr || out == nullptr) {
    set_error("null argument");
    return AIRICE_EINVAL;
  }
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) {
    set_error("cannot open atmosphere file '%s'", path);
    return AIRICE_EIO;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  return airice_atmosphere_parse(s.data(), s.size(), variant, out);
}

int airice_grid_init(airice_grid* g, double depth_cm, double ice_cm, double height_step,
                     double start_angle, double stop_angle, double angle_step) {
  if (g == nullptr || !(height_step > 0) || !(angle_step > 0) || !(stop_angle >= start_angle)) {
    set_error("invalid grid arguments");
    return AIRICE_EINVAL;
  }
  // MakeRayTracingTable (.cc:2021-2061)
  g->in_ice = depth_cm < 0 ? 1 : 0;
  g->depth_m = depth_cm / 100;
  g->ice_m = ice_cm / 100;
  g->start_height = 100000;
  g->stop_height = g->in_ice ? g->ice_m : g->ice_m + g->depth_m;
  g->height_step = height_step;
  // the reference's int conversions (.cc:2046, :15) of the step counts; counts beyond int range
  // (or NaN) would be undefined there and are rejected here
  const double hs = std::floor((g->start_height - g->stop_height) / height_step) + 1;
  const double as = std::floor((stop_angle - start_angle) / angle_step) + 1;
  if (!(hs >= 1 && hs <= 2147483647.0) || !(as >= 1 && as <= 2147483647.0)) {
    set_error("empty grid or step counts beyond int range (%g x %g)", hs, as);
    return AIRICE_EINVAL;
  }
  g->height_steps = (int32_t)hs;
  g->start_angle = start_angle;
  g->stop_angle = stop_angle;
  g->angle_step = angle_step;
  g->angle_steps = (int32_t)as;
  if (g->height_steps < 1 || g->angle_steps < 1) {
    set_error("empty grid");
    return AIRICE_EINVAL;
  }
  // The reference skips rows whose (unforced) AirTxHeight is not > 0 (.cc:2081-2082); heights
  // fall with the row index, so the kept rows are a prefix
  int32_t rows = g->height_steps;
  while (rows > 0 && !(g->start_height - g->height_step * (rows - 1) > 0)) --rows;
  g->table_rows = rows;
  return AIRICE_OK;
}

uint64_t airice_table_checksum(const float* h_table, size_t ld, size_t n_rays) {
  uint64_t r = 0x5DEECE66Dull ^ n_rays;
  if (h_table == nullptr) return r;
  for (int c = 0; c < AIRICE_TABLE_COLUMNS; ++c)
    r = bytes_hash(reinterpret_cast<const unsigned char*>(h_table + (size_t)c * ld),
                   n_rays * sizeof(float), r + (uint64_t)c);
  return r;
}

int airice_table_save(const char* path, const airice_medium* m, const airice_grid* g,
                      const float* h_table, size_t ld, size_t n_rays) {
  if (path == nullptr || m == nullptr || g == nullptr || (h_table == nullptr && n_rays > 0) ||
      ld < n_rays) {
    set_error("table_save: null argument or column stride < n_rays");
    return AIRICE_EINVAL;
  }
  unsigned char hdr[AIRICE_TABLE_FILE_HEADER] = {};
  std::memcpy(hdr, kTableMagic, 8);
  uint32_t version = kTableVersion, hbytes = AIRICE_TABLE_FILE_HEADER,
           cols = AIRICE_TABLE_COLUMNS;
  uint64_t n = n_rays, sum = airice_table_checksum(h_table, ld, n_rays);
  HeaderIO io{hdr, 8, true};
  io.f(version);
  io.f(hbytes);
  io.f(cols);
  io.skip(12);
  io.f(n);
  io.f(sum);
  airice_medium mc = *m;
  airice_grid gc = *g;
  medium_io(io, mc);
  grid_io(io, gc);
  // write a sibling temporary and rename it into place: a reader never sees a half-written file
  const std::string tmp = std::string(path) + ".part";
  FileCloser fc{std::fopen(tmp.c_str(), "wb")};
  if (fc.f == nullptr) {
    set_error("table_save: cannot create '%s'", tmp.c_str());
    return AIRICE_EIO;
  }
  bool ok = std::fwrite(hdr, 1, sizeof(hdr), fc.f) == sizeof(hdr);
  for (int c = 0; ok && c < AIRICE_TABLE_COLUMNS && n_rays > 0; ++c)
    ok = std::fwrite(h_table + (size_t)c * ld, sizeof(float), n_rays, fc.f) == n_rays;
  ok = (std::fclose(fc.f) == 0) && ok;
  fc.f = nullptr;
  if (!ok || std::rename(tmp.c_str(), path) != 0) {
    std::remove(tmp.c_str());
    set_error("table_save: writing '%s' failed", path);
    return AIRICE_EIO;
  }
  return AIRICE_OK;
}

int airice_table_file_read_info(const char* path, airice_table_file_info* info) {
  if (path == nullptr || info == nullptr) {
    set_error("table_file_read_info: null argument");
    return AIRICE_EINVAL;
  }
  FileCloser fc{std::fopen(path, "rb")};
  if (fc.f == nullptr) {
    set_error("table file: cannot open '%s'", path);
    return AIRICE_EIO;
  }
  unsigned char hdr[AIRICE_TABLE_FILE_HEADER];
  if (std::fread(hdr, 1, sizeof(hdr), fc.f) != sizeof(hdr) || std::memcmp(hdr, kTableMagic, 8)) {
    set_error("table file '%s': not an airice table file", path);
    return AIRICE_EINVAL;
  }
  uint32_t version = 0, hbytes = 0, cols = 0;
  uint64_t n = 0, sum = 0;
  HeaderIO io{hdr, 8, false};
  io.f(version);
  io.f(hbytes);
  io.f(cols);
  io.skip(12);
  io.f(n);
  io.f(sum);
  if (version != kTableVersion || hbytes != AIRICE_TABLE_FILE_HEADER ||
      cols != AIRICE_TABLE_COLUMNS) {
    set_error("table file '%s': unsupported version %u / header %u / columns %u", path, version,
              hbytes, cols);
    return AIRICE_EINVAL;
  }
  std::memset(info, 0, sizeof(*info));
  medium_io(io, info->medium);
  grid_io(io, info->grid);
  info->n_rays = n;
  info->checksum = sum;
  // the body must hold exactly the 11 columns the header announces
  if (std::fseek(fc.f, 0, SEEK_END) != 0) {
    set_error("table file '%s': cannot seek", path);
    return AIRICE_EIO;
  }
  const long long len = (long long)ftello(fc.f);
  const unsigned long long want =
      (unsigned long long)AIRICE_TABLE_FILE_HEADER + (unsigned long long)AIRICE_TABLE_COLUMNS * 4ull * n;
  if (n > (1ull << 56) || len < 0 || (unsigned long long)len != want) {
    set_error("table file '%s': %lld bytes, the header announces %llu", path, len, want);
    return AIRICE_EINVAL;
  }
  return AIRICE_OK;
}

int airice_table_load(const char* path, const airice_medium* expect, float* h_table, size_t ld,
                      airice_table_file_info* info) {
  airice_table_file_info fi;
  int rc = airice_table_file_read_info(path, &fi);
  if (rc != AIRICE_OK) return rc;
  if (expect != nullptr && !same_medium(*expect, fi.medium)) {
    set_error("table file '%s' was traced in another medium (atmosphere / ice model / variant)",
              path);
    return AIRICE_EINVAL;
  }
  const size_t n = (size_t)fi.n_rays;
  if ((h_table == nullptr && n > 0) || ld < n) {
    set_error("table_load: null table or column stride %zu < %zu entries", ld, n);
    return AIRICE_EINVAL;
  }
  FileCloser fc{std::fopen(path, "rb")};
  if (fc.f == nullptr || std::fseek(fc.f, AIRICE_TABLE_FILE_HEADER, SEEK_SET) != 0) {
    set_error("table file: cannot open '%s'", path);
    return AIRICE_EIO;
  }
  for (int c = 0; c < AIRICE_TABLE_COLUMNS && n > 0; ++c) {
    if (std::fread(h_table + (size_t)c * ld, sizeof(float), n, fc.f) != n) {
      set_error("table file '%s': short read in column %d", path, c);
      return AIRICE_EIO;
    }
  }
  if (airice_table_checksum(h_table, ld, n) != fi.checksum) {
    set_error("table file '%s': checksum mismatch (corrupt file)", path);
    return AIRICE_EIO;
  }
  if (info != nullptr) *info = fi;
  return AIRICE_OK;
}

}  // extern "C"
