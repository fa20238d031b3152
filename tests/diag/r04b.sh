# which caller-keypoint test stops (dual descriptor), each under its own limit
set -o pipefail
mkdir -p gpurun_out
T="tests/test_gpu_parity.py -m gpu -v --timeout 60 --timeout-method thread -s"
timeout -k 10 100 python -u -m pytest $T -k "detected_keypoints_fed_back" 2>&1 | tee gpurun_out/pytest_b1.log | tail -15; echo "rc=$?"
