# Round-4 re-trim check: the trim / re-trim parity tests, the per-round phase timing (HG_TIMING
# build), the trim-batch latency probe and the bench line's re-trim secondary.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "${K:-trim or retrim or azimuth}" > gpurun_out/r04_retrim_tests.txt 2>&1
rc=$?; tail -4 gpurun_out/r04_retrim_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
HELIGYM_AMD_LIB=$PWD/build/variants/timing.so timeout -k 10 120 python scripts/retrim_timing.py > gpurun_out/r04_retrim_timing.txt 2>&1 || { echo "timing failed"; tail -5 gpurun_out/r04_retrim_timing.txt; exit 3; }
cat gpurun_out/r04_retrim_timing.txt | grep -v amdgpu.ids
timeout -k 10 200 python scripts/retrim_probe.py > gpurun_out/r04_retrim_probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r04_retrim_probe.txt; exit 4; }
grep -v amdgpu.ids gpurun_out/r04_retrim_probe.txt
timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline --no-parity > gpurun_out/r04_bench_retrim.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r04_bench_retrim.log; exit 5; }
tail -1 gpurun_out/r04_bench_retrim.log > gpurun_out/r04_bench_retrim.json
python scripts/bench_brief.py gpurun_out/r04_bench_retrim.json
