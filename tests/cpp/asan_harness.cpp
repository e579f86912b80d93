// Sanitizer harness (ASan/UBSan CPU builds), built by `make asan` with
// -fsanitize=address,undefined -fno-sanitize-recover=all and run by tests/test_asan.py.
//
// It drives the host code of libairice.so -- the GDAS parse and grid set-up (airice_host.cpp),
// the namespace readers of the C++ drop-ins (compat_common.h), the host table lookup that the
// scalar _Table / FindClosest* / GetParValues exports run (airice_lookup.hpp, both the column
// path and the packed-record path) -- and the oracle (oracle/airice_oracle.c), on the real
// Atmosphere.dat, on hostile atmosphere texts (empty, truncated at many offsets, garbage and
// non-finite tokens, a profile with too many layers) and on edge lookups (NaN, H <= 0, heights
// outside the table, D = 0, D beyond every THD).  The reference has known undefined behaviour
// next to these paths (MultiRayAirIceRefraction.cc:668, :1802, the lookup's out-of-table reads);
// the library's versions must run clean.  Prints one JSON object.
//
// usage: asan_harness Atmosphere.dat table.bin
//   table.bin: int64 n, double stop_h, double step_h, int32 hsteps, int32 asteps, then 11 x n
//              float32 columns (an oracle-built table, tests/test_asan.py)
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "airice.h"
#include "airice_lookup.hpp"
#include "compat_common.h"

extern "C" {
#include "airice_oracle.h"
}

namespace {

std::string read_file(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::ostringstream s;
  s << f.rdbuf();
  return s.str();
}

// every parser on one text: rc / layers of each (no crash, no UB is the test)
void parse_all(const std::string& text, int& rc_lib, int& rc_oracle, int& layers_ns) {
  airice_medium m;
  rc_lib = airice_atmosphere_parse(text.data(), text.size(), AIRICE_VARIANT_MULTIRAY, &m);
  if (rc_lib == AIRICE_OK && !(m.max_layers >= 1 && m.max_layers <= 4 && std::isfinite(m.N0))) {
    // a parse that succeeds must hand out a usable medium
    std::fprintf(stderr, "parse accepted an unusable medium\n");
    std::abort();
  }
  double ATMLAY[5], abc[5][3];
  std::vector<std::vector<double>> h, n, ln;
  airice_compat::read_atm_par(text, ATMLAY, abc);
  layers_ns = airice_compat::read_nh(text, ATMLAY, h, n, ln);
  or_medium om;
  rc_oracle = or_parse_atmosphere(text.data(), text.size(), 3.1415927, &om);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: asan_harness Atmosphere.dat table.bin\n");
    return 2;
  }
  const std::string atm = read_file(argv[1]);
  std::printf("{\n");

  // ---- atmosphere parse: the real file, then hostile texts ----------------------------------
  int rl, ro, ln;
  parse_all(atm, rl, ro, ln);
  std::printf("\"real\": [%d, %d, %d],\n", rl, ro, ln);
  std::vector<std::string> hostile = {
      "", "\n", "\n\n\n\n\n\n", "1 2 3 4 5\n", "garbage\nnot numbers at all\n\n\n\n\nx y\n",
      "0 1 2 3 4\n1 1 1 1 1\n2 2 2 2 2\n3 3 3 3 3\n\nnan nan\ninf inf\n-inf 5\n1e308 1e308\n",
      std::string(100000, '9') + "\n",
      // a profile whose heights run past every ATMLAY bound (more layers than the 5 bounds hold)
      "0 1000 2000 3000 4000\n1 1 1 1 1\n1 1 1 1 1\n1000 1000 1000 1000 1000\n\n"};
  {
    std::string many;
    for (int h = 0; h < 20000000; h += 250000) many += std::to_string(h / 100) + " 1.0003\n";
    hostile.push_back("0 1000 2000 3000 4000\n1 1 1 1 1\n1 1 1 1 1\n1000 1000 1000 1000 1000\n\n" +
                      many);
  }
  // truncations of the real file: the header, the first profile lines, and spread offsets
  for (size_t cut = 0; cut < 1200 && cut < atm.size(); cut += 7) hostile.push_back(atm.substr(0, cut));
  for (size_t k = 1; k < 40; ++k) hostile.push_back(atm.substr(0, atm.size() * k / 40));
  // binary junk spliced into the profile
  {
    std::string j = atm.substr(0, 5000);
    for (size_t i = 600; i < j.size(); i += 97) j[i] = (char)(i * 131);
    hostile.push_back(j + atm.substr(5000, 20000));
  }
  int lib_ok = 0, oracle_ok = 0;
  for (const std::string& t : hostile) {
    parse_all(t, rl, ro, ln);
    lib_ok += rl == AIRICE_OK;
    oracle_ok += ro == 0;
  }
  std::printf("\"hostile\": [%zu, %d, %d],\n", hostile.size(), lib_ok, oracle_ok);

  // ---- grid set-up edge arguments ----------------------------------------------------------
  {
    const double args[][6] = {{-20000, 300000, 10, 90.1, 180, 0.1},   // the reference default
                              {-20000, 300000, 0, 90.1, 180, 0.1},    // zero step
                              {-20000, 300000, -5, 90.1, 180, 0.1},   // negative step
                              {-20000, 300000, NAN, 90.1, 180, 0.1},  // NaN step
                              {-20000, 300000, 1e-300, 90.1, 180, 0.1},  // counts beyond int
                              {-20000, 300000, 10, 180, 90, 0.1},     // reversed angles
                              {-20000, 300000, 10, 90.1, 180, 1e-300},
                              {5000, -2000000, 3000, 90.1, 180, 1},   // Tx rows <= 0 (.cc:2082)
                              {0, 1e12, 10, 90.1, 180, 1}};          // ice above the Tx start
    std::printf("\"grid\": [");
    for (size_t i = 0; i < sizeof(args) / sizeof(args[0]); ++i) {
      airice_grid g;
      const int rc = airice_grid_init(&g, args[i][0], args[i][1], args[i][2], args[i][3],
                                      args[i][4], args[i][5]);
      std::printf("[%d, %d, %d, %d]%s", rc, rc == 0 ? g.height_steps : 0,
                  rc == 0 ? g.angle_steps : 0, rc == 0 ? g.table_rows : 0,
                  i + 1 < sizeof(args) / sizeof(args[0]) ? ", " : "");
    }
    std::printf("],\n");
  }

  // ---- host table lookup: column path and packed path vs the oracle -------------------------
  std::ifstream tf(argv[2], std::ios::binary);
  int64_t n = 0;
  double stop_h = 0, step_h = 0;
  int32_t hsteps = 0, asteps = 0;
  tf.read(reinterpret_cast<char*>(&n), 8);
  tf.read(reinterpret_cast<char*>(&stop_h), 8);
  tf.read(reinterpret_cast<char*>(&step_h), 8);
  tf.read(reinterpret_cast<char*>(&hsteps), 4);
  tf.read(reinterpret_cast<char*>(&asteps), 4);
  std::vector<float> cols((size_t)n * AIRICE_TABLE_COLUMNS);
  tf.read(reinterpret_cast<char*>(cols.data()), (std::streamsize)(sizeof(float) * cols.size()));
  if (!tf || n <= 0 || asteps <= 0) {
    std::fprintf(stderr, "bad table file\n");
    return 2;
  }
  airice::LkTable T;
  for (int c = 0; c < AIRICE_TABLE_COLUMNS; ++c) T.col[c] = cols.data() + (size_t)c * n;
  T.e = nullptr;
  T.rows = 0;
  T.n = n;
  T.stop_h = stop_h;
  T.step_h = step_h;
  T.hsteps = hsteps;
  T.asteps = asteps;
  // the packed copy airice_lookup_pack makes on the device, built here with the same layout and
  // the same row-record fold (lk_row_fold)
  std::vector<float> packed(AIRICE_LOOKUP_PACK_FLOATS(n, asteps) + 4);
  float* e = packed.data();
  while ((reinterpret_cast<uintptr_t>(e) & 15) != 0) ++e;  // 16-byte aligned records
  for (int64_t i = 0; i < n; ++i)
    airice::lk_pair_fold(T.col, n, i, e + (size_t)AIRICE_LOOKUP_ENTRY_FLOATS * i);
  airice::LkTable P = T;
  P.e = e;
  P.rows = n / asteps;
  for (int64_t r = 0; r < P.rows; ++r)
    airice::lk_row_fold(P, r, e + AIRICE_LOOKUP_ROWS_OFFSET(n) + (size_t)r * AIRICE_LOOKUP_ROW_FLOATS);
  // the angle vector (column 4 of the first row; the harness's tables are MakeRayTracingTable's,
  // so every row has it -- checked here as the pack checks it)
  float* ang = e + airice::lk_angles_offset(n, asteps);
  bool ang_ok = true;
  for (int64_t j = 0; j < asteps; ++j) ang[j] = j < n ? T.col[4][j] : NAN;
  for (int64_t i = 0; i < n; ++i)
    ang_ok = ang_ok && airice::lk_bits_i(T.col[4][i]) == airice::lk_bits_i(T.col[4][i % asteps]);
  P.ang = ang_ok ? ang : nullptr;
  or_lookup_table ot;
  for (int c = 0; c < 11; ++c) ot.col[c] = T.col[c];
  ot.n = (long)n;
  ot.LoopStopHeight = stop_h;
  ot.HeightStepSize = step_h;
  ot.TotalHeightSteps = hsteps;
  ot.TotalAngleSteps = asteps;
  or_medium om;
  or_parse_atmosphere(atm.data(), atm.size(), 3.1415927, &om);

  const double hmax = T.col[0][0], hmin = T.col[0][n - 1];
  std::vector<std::pair<double, double>> qs = {
      {NAN, 1000}, {5000, NAN}, {NAN, NAN}, {0, 1000}, {-50, 1000}, {hmax, 0}, {hmin, 0},
      {hmax + 1e-3, 100}, {hmin - 1e-3, 100}, {hmax * 10, 100}, {5000, 1e9}, {5000, 1e300},
      {hmin + 1e-7, 50}, {hmax - 1e-7, 5000}, {1e300, 1e300}, {-1e300, -1e300}, {5000, -100},
      {INFINITY, 100}, {5000, INFINITY}};
  uint64_t s = 0x9E3779B97F4A7C15ull;
  auto u = [&s]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return (double)(s >> 11) * 0x1p-53;
  };
  for (int i = 0; i < 3000; ++i) qs.push_back({hmin + (hmax - hmin) * u(), 60000.0 * u()});
  for (int i = 0; i < 200 && n > 1; ++i) {  // queries exactly on table entries (.cc:1212 branch)
    const int64_t k = (int64_t)(u() * (double)(n - 1));
    qs.push_back({T.col[0][k], T.col[1][k]});
  }
  int n_fallback = 0, n_col_vs_packed = 0, n_vs_oracle = 0, n_checked = 0, n_unpinned = 0;
  const double d2r = 3.1415927 / 180.0;
  for (const auto& q : qs) {
    double o1[9], o2[9], oref[9];
    bool g1 = false, g2 = false;
    int f1 = 0, f2 = 0, fref = 0;
    // cm arguments as the reference's _Table takes them; the library divides by 100 (.cc:1307)
    const double src_cm = q.first * 100, dist_cm = q.second * 100;
    const bool fb1 = airice::lk_query(T, src_cm / 100, dist_cm / 100, d2r, o1, &g1, f1);
    const bool fb2 = airice::lk_query(P, src_cm / 100, dist_cm / 100, d2r, o2, &g2, f2);
    const int ok_ref = or_table_lookup(&om, &ot, src_cm, dist_cm, -20000.0, 300000.0, oref, &fref);
    n_unpinned += (f1 & AIRICE_LOOKUP_UNPINNED) != 0;
    if (fb1 || fb2) {  // the minimizer fallback runs on the GPU: flags must agree
      n_fallback++;
      if (fb1 != fb2) n_col_vs_packed++;
      continue;
    }
    if (g1 != g2 || std::memcmp(o1, o2, sizeof(o1)) != 0) n_col_vs_packed++;
    n_checked++;
    bool same = (g1 == (ok_ref != 0));
    for (int c = 0; c < 9; ++c)
      if (!(o1[c] == oref[c] || (std::isnan(o1[c]) && std::isnan(oref[c])))) same = false;
    if (!same && (fref & OR_LK_FALLBACK) == 0) {
      if (n_vs_oracle < 5 && std::getenv("ASAN_HARNESS_VERBOSE") != nullptr) {
        std::fprintf(stderr, "mismatch H=%.17g D=%.17g ok %d/%d fl %d/%d\n", q.first, q.second,
                     (int)g1, ok_ref, f1, fref);
        for (int c = 0; c < 9; ++c) std::fprintf(stderr, "  %d %.17g %.17g\n", c, o1[c], oref[c]);
      }
      n_vs_oracle++;
    }
  }
  std::printf("\"lookup\": {\"queries\": %zu, \"checked\": %d, \"fallback\": %d, "
              "\"unpinned\": %d, \"col_vs_packed_mismatch\": %d, \"vs_oracle_mismatch\": %d},\n",
              qs.size(), n_checked, n_fallback, n_unpinned, n_col_vs_packed, n_vs_oracle);

  // ---- table files: save / load round trip, then damaged files ------------------------------
  {
    airice_medium med;
    airice_atmosphere_parse(atm.data(), atm.size(), AIRICE_VARIANT_MULTIRAY, &med);
    airice_grid g;
    airice_grid_init(&g, -20000.0, 300000.0, step_h, 92.0, 180.0, 1.0);
    const std::string path = std::string(argv[2]) + ".airtbl";
    int rc_save = airice_table_save(path.c_str(), &med, &g, cols.data(), (size_t)n, (size_t)n);
    const size_t ld = (size_t)n + 7;  // a wider destination stride
    std::vector<float> back(ld * AIRICE_TABLE_COLUMNS, -1.0f);
    airice_table_file_info info;
    int rc_load = airice_table_load(path.c_str(), &med, back.data(), ld, &info);
    bool same = rc_save == 0 && rc_load == 0 && info.n_rays == (uint64_t)n &&
                info.grid.angle_steps == g.angle_steps && info.medium.max_layers == med.max_layers;
    for (int c = 0; same && c < AIRICE_TABLE_COLUMNS; ++c)
      same = std::memcmp(back.data() + (size_t)c * ld, cols.data() + (size_t)c * n,
                         sizeof(float) * (size_t)n) == 0;
    // another medium (the pythonwrapper's pi) is refused
    airice_medium other = med;
    other.pi = 4.0 * std::atan(1.0);
    const int rc_other = airice_table_load(path.c_str(), &other, back.data(), ld, nullptr);
    // damaged copies: truncated at several lengths, a flipped body byte, a flipped magic byte, an
    // inflated entry count, another version; every one must be refused without a fault
    const std::string img = read_file(path.c_str());
    std::vector<std::string> bad;
    for (size_t cut : {(size_t)0, (size_t)7, (size_t)100, (size_t)511, (size_t)512,
                       img.size() / 2, img.size() - 1})
      bad.push_back(img.substr(0, cut));
    std::string b = img;
    b[AIRICE_TABLE_FILE_HEADER + 4 * (size_t)n + 3] ^= 0x10;
    bad.push_back(b);
    b = img;
    b[0] ^= 1;
    bad.push_back(b);
    b = img;
    b[32 + 7] = 0x7f;  // n_rays: ~2^62 entries
    bad.push_back(b);
    b = img;
    b[8] = 2;  // version
    bad.push_back(b);
    b = img + "x";  // trailing byte
    bad.push_back(b);
    int rejected = 0;
    const std::string bpath = path + ".bad";
    for (const auto& s : bad) {
      std::ofstream(bpath, std::ios::binary).write(s.data(), (std::streamsize)s.size());
      rejected += airice_table_load(bpath.c_str(), nullptr, back.data(), ld, nullptr) != 0;
    }
    std::remove(bpath.c_str());
    std::remove(path.c_str());
    std::printf("\"table_file\": [%d, %d, %zu, %d],\n", same ? 1 : 0, rc_other != 0 ? 1 : 0,
                bad.size(), rejected);
  }

  // ---- the oracle's own ray / solve paths on edge geometries ---------------------------------
  {
    double d[18], dm[17], dp[15], a10[10];
    const double ray_args[][3] = {{90.0, 100000, -200}, {180, 3000, -200}, {90.1, 3000.5, -200},
                                  {170, 1e6, -200},     {120, 5000, 100},  {NAN, 5000, -200}};
    for (const auto& a : ray_args) or_ray_solution(&om, a[0], a[1], 3000, a[2], a[2] < 0, d);
    const double q[][3] = {{5000, 1000, -200}, {3000.5, 0, -5},     {100000, 50000, -300},
                           {3100, 1e6, -1},    {3500, 10, 200},     {NAN, 100, -10},
                           {5000, NAN, -10},   {2000, 100, -10},    {1e9, 1e9, -10}};
    int st = 0;
    for (const auto& x : q) {
      const double thR = or_straight_angle(&om, x[0], x[1], 3000, x[2]);
      st |= or_air2ice(&om, x[0], x[1], 3000, x[2], thR, dm);
      st |= or_py_air2ice(&om, x[0], x[1], 3000, x[2], thR, dp);
      or_py_trace_ice_to_air(&om, x[2], 3000, x[0], x[1], a10);
    }
    std::printf("\"oracle_paths\": %d\n", st >= 0 ? 1 : 0);
  }
  std::printf("}\n");
  return 0;
}
