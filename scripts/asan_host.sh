# Host-code sanitizer run (CPU only; GPU sanitizers are not available on the pool): build the
# library with AddressSanitizer + UBSan on the host side of both translation units, then run the
# host tests (trim, config, loaders, error paths) against it.
set -eu
cd "$(dirname "$0")/.."
D=build/asan; mkdir -p $D
F="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -fno-hip-fp32-correctly-rounded-divide-sqrt -fgpu-flush-denormals-to-zero"
S="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined"
/opt/rocm/bin/hipcc $F -ffp-contract=on $S -c -o $D/a.o heli-gym_amd/csrc/heligym_amd.hip
/opt/rocm/bin/hipcc $F -ffp-contract=off $S -c -o $D/b.o heli-gym_amd/csrc/retrim.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -fsanitize=address -fsanitize=undefined -shared-libsan \
    -o $D/libheligym_amd.so $D/a.o $D/b.o
RT=$(find /opt/rocm/lib/llvm -name "libclang_rt.asan-x86_64.so" | head -1)
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    HELIGYM_AMD_LIB=$PWD/$D/libheligym_amd.so \
    python -m pytest tests/test_abi_host.py tests/test_airframe_loader.py -q -m "not gpu" -k "not plain_c" -p no:cacheprovider
