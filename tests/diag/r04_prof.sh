# Round 4 profiles: kernel trace + calibrated HBM counters of the headline, C4 trace, feature
# kernel counters (descriptor / orientation / extremum), C2 trace
set -o pipefail
TAG=${1:-r04a}
mkdir -p gpurun_out
timeout -k 10 900 bash tests/profile_kernels.sh "$TAG" > gpurun_out/prof_$TAG.log 2>&1 && echo profile ok && \
timeout -k 10 400 bash tests/pmc_desc.sh "$TAG" > gpurun_out/pmc_desc_$TAG.log 2>&1 && echo pmc desc ok && \
timeout -k 10 300 bash tests/profile_c2.sh "$TAG" > gpurun_out/prof_c2_$TAG.log 2>&1 && echo c2 ok
tail -5 gpurun_out/prof_$TAG.log
