# round 2, run w: destination-major write-many calibration vs the chunk-major synthetic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02w
timeout -k 10 120 ./tools/store_peak3 > gpurun_out/r02w/peak3.json && cat gpurun_out/r02w/peak3.json && \
timeout -k 10 120 ./tools/store_peak4 > gpurun_out/r02w/peak4.json && cat gpurun_out/r02w/peak4.json
