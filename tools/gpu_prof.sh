#!/bin/bash
# Profile session: kernel microbench, then rocprofv3 kernel-trace stats of a short bench,
# then a separate PMC pass (FETCH_SIZE / WRITE_SIZE) on the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r1}
BARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu --no-solve}
run() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 30 "gpurun_out/$name.log"
    return $rc
}
if [[ ${STEPS:-kbench,trace,pmc} == *kbench* ]]; then
    run kbench 300 python tools/kbench.py || exit $?
fi
if [[ ${STEPS:-kbench,trace,pmc} == *trace* ]]; then
    run prof_trace 600 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/prof_$TAG -o trace -- python bench.py $BARGS || exit $?
fi
if [[ ${STEPS:-kbench,trace,pmc} == *pmc* ]]; then
    run prof_fetch 600 rocprofv3 --kernel-trace -T --pmc FETCH_SIZE -f csv -d gpurun_out/prof_${TAG}_fetch -o pmc -- python bench.py $BARGS || exit $?
    run prof_write 600 rocprofv3 --kernel-trace -T --pmc WRITE_SIZE -f csv -d gpurun_out/prof_${TAG}_write -o pmc -- python bench.py $BARGS || exit $?
fi
find gpurun_out -name "*stats*.csv" | head
