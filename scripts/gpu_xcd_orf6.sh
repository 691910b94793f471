set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/xcd
MAGOT_LIB=$PWD/scripts/lib_xcd.so timeout -k 10 300 python -u -m pytest tests -m "gpu and not slow" -k "orf6" -x -q --timeout 120 --timeout-method thread > gpurun_out/xcd/pytest.log 2>&1 || { tail -30 gpurun_out/xcd/pytest.log; exit 1; }
tail -1 gpurun_out/xcd/pytest.log
bash scripts/ab_multi.sh "scripts/lib_base.so scripts/lib_xcd.so scripts/lib_xcdplain.so" --config C5 --steps 30 --warmup 10 && KERNEL=orf6_kernel BENCH_ARGS="--config C5" bash scripts/ab_write_size.sh "scripts/lib_base.so scripts/lib_xcd.so scripts/lib_xcdplain.so"
