"""Per-rank entry for the CPU test of bench.py's self-launch (test infrastructure only):
bench.self_launch starts ``torch.distributed.run --nproc-per-node N`` on this script instead of
bench.py, and each rank runs bench.main() over gloo with the CPU rehearsal backend
(tests/bench_rehearsal.py) in place of the HIP kernels."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    os.environ["AIRICE_DIST_BACKEND"] = "gloo"
    import bench
    from tests.bench_rehearsal import CpuRehearsalBackend
    bench.main(sys.argv[1:], make_backend=CpuRehearsalBackend)
