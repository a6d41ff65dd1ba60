# Overlapped next-step re-trim: its bitwise tests with the re-trim / azimuth / next-step tests, the
# re-trim cost by mode, and the short-window timing probe.  Each GPU step has its own limit.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "${K:-overlap or trim or retrim or azimuth or next_step or rollout}" > gpurun_out/r04_ov_tests.txt 2>&1
rc=$?; tail -4 gpurun_out/r04_ov_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ $rc -eq 1 ] && exit 1
timeout -k 10 200 python scripts/retrim_modes.py > gpurun_out/r04_retrim_modes.txt 2>&1 || { echo "modes failed"; tail -5 gpurun_out/r04_retrim_modes.txt; exit 4; }
grep -v amdgpu.ids gpurun_out/r04_retrim_modes.txt
timeout -k 10 200 python scripts/r04_window_probe.py > gpurun_out/r04_window_probe.txt 2>&1 || { echo "window probe failed"; tail -5 gpurun_out/r04_window_probe.txt; exit 5; }
grep -v amdgpu.ids gpurun_out/r04_window_probe.txt
OV=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ovtrace1 -o run -- python3 scripts/r04_ov_trace.py > gpurun_out/ovtrace1.txt 2>&1 || { echo "ov trace failed"; exit 6; }
grep -h "us/step" gpurun_out/ovtrace1.txt
