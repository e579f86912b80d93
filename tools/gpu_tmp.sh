set -o pipefail
bash tools/gpu_lib_pmc.sh gpurun_out/r04e ab/lib_r03.so ab/lean1.so ab/pairs1.so
