"""The guarded bisection's closed-form lean run (airiceraytracing_amd/csrc/airice_lean.hpp) against
its step-by-step form on fuzzed brackets built the way solve_root builds them (tests/cpp/lean_check.cpp,
g++ -ffp-contract=off): the same lo, hi, step count and exit, bit for bit, on every bracket the
closed form accepts.  The GPU side of the same check is tests/test_gpu_bisect_replay.py (roots and
status bits of the guarded solver against the every-midpoint form)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_closed_form_lean_run_matches_the_steps(tmp_path):
    exe = str(tmp_path / "lean_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off",
                    "-I" + os.path.join(ROOT, "airiceraytracing_amd", "csrc"), "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "lean_check.cpp")], check=True)
    r = subprocess.run([exe, "3000000"], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
    f = dict(zip(r.stdout.split()[0::2], map(int, r.stdout.split()[1::2])))
    assert f["mismatches"] == 0
    # the probe's steps in closed form: bit-identical to the loop on every case
    assert f["probe_mismatches"] == 0 and f["probe_cases"] > 0.2 * f["cases"]
    # most brackets take the closed form, and a good share of the runs end the solve
    assert f["closed"] > 0.6 * f["cases"] and f["done"] > 0.1 * f["closed"]
