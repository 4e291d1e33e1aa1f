#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Each GPU step has its own time
# limit; a crash/timeout (exit >= 124 or signal) ends the script without further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
    return $rc
}
STEPS=${STEPS:-pytest,smoke,bench}
if [[ $STEPS == *pytest* ]]; then
    run pytest_gpu 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-}
    rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [[ $STEPS == *smoke* ]]; then
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [[ $STEPS == *bench* ]]; then
    run bench 600 python bench.py ${BENCH_ARGS:-} || exit $?
fi
