#!/bin/bash
# The one GPU-box runner (replaces the per-session tools/gpu_r*.sh scripts).
#
#   STEPS="pytest,smoke,bench" O=gpurun_out/r4a bash tools/gpu.sh
#
# Every step runs under its own `timeout -k 10`, writes its log under $O, and a failure
# (non-zero status, a signal, a time limit) ends the script: no GPU step runs after a
# crashed or hung one.  Steps (in the order given):
#   pytest        the whole GPU suite                     PYTEST_K="-k expr" narrows it
#   pytest:FILE   one test file (tests/FILE)
#   smoke         __graft_entry__.smoke()
#   bench         python bench.py $BENCH_ARGS             (the driver's command by default)
#   gloo4         CGP_BENCH_BACKEND=gloo bench.py --gpus 4 (the launcher, 4 ranks, 1 GPU)
#   failleg       bench.py with CGP_BENCH_FAIL_LEG=mnist_as_tf (the line must still print)
#   tile4096      bench.py --tile 4096 --steps 2 (no OOM in the stencil probe)
#   trace:CFG     rocprofv3 --kernel-trace --stats over bench.py --config CFG
#   pmc           PMC passes (tools/pmc.sh; PMC_CFGS) summarised into $O/net_pmc.json
#   fullscale     tools/fullscale.py $FS_ARGS
#   py:SCRIPT     python SCRIPT (a probe under tools/)
#   ab            netbench (NB_ARGS) for each build in $AB: "cur" = lib/libcnngp.so, any other
#                 name = cnn-gp_amd/lib/ab/lib_NAME.so (tools/build_variant.sh); AB_REPS rounds;
#                 AB_TEST=1 runs each variant's whole-network parity tests first; AB_TOOL
#                 times another script (e.g. tools/stencil_once.py); a NAME=VALUE
#                 entry runs the current library with that environment variable
#   envtest       pytest $PYTEST_ARGS with the environment ENVTEST="NAME=VALUE ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/run}
mkdir -p "$O"

step() {   # name limit cmd...
    local name=$1 t=$2; shift 2
    local t0=$SECONDS
    # a bench.py run writes its full result beside its log (one file per step: a later
    # bench step must not overwrite an earlier one's)
    CGP_BENCH_FULL_OUT="$PWD/$O/${name}_full.json" timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc ($((SECONDS - t0)) s)"
    if [ $rc -ne 0 ]; then tail -n 40 "$O/$name.log"; exit $rc; fi
}

line() {   # the bench JSON line of a log, summarised
    python3 tools/bench_summary.py "$1"
}

IFS=',' read -ra LIST <<< "${STEPS:-pytest,smoke,bench}"
for s in "${LIST[@]}"; do
    case $s in
    pytest)
        step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
            --timeout-method thread ${PYTEST_K:-}
        tail -n 1 "$O/pytest.log" ;;
    pytest:*)
        f=${s#pytest:}
        step "pytest_${f%.py}" 900 python -u -m pytest "tests/$f" -x -v -s --timeout 600 \
            --timeout-method thread ${PYTEST_K:-}
        grep -E "passed|failed|worst|bit-equal" "$O/pytest_${f%.py}.log" | tail -n 12 ;;
    smoke)
        step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
        tail -n 1 "$O/smoke.log" ;;
    bench)
        step bench 1200 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5}
        line "$O/bench.log" ;;
    gloo4)
        CGP_BENCH_BACKEND=gloo step gloo4 900 python bench.py --gpus 4 --steps 2 --warmup 1 \
            --no-cpu --no-f32 --no-fullscale-f32 --fullscale-n 16384 --cifar10-n 16384 \
            --fullscale-m 4096
        line "$O/gloo4.log" ;;
    failleg)
        CGP_BENCH_FAIL_LEG=mnist_as_tf step failleg 600 python bench.py --steps 2 \
            --warmup 1 --no-cpu --no-f32 --no-fullscale --no-fullscale-cifar10 --no-cifar10
        line "$O/failleg.log" ;;
    tile4096)
        step tile4096 900 python bench.py --tile 4096 --steps 2 --warmup 1 --no-cpu \
            --no-f32 --no-fullscale --no-fullscale-cifar10 --no-second --no-cifar10 --no-dropin
        line "$O/tile4096.log" ;;
    trace:*)
        cfg=${s#trace:}
        step "trace_$cfg" 600 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/trace_$cfg" \
            -o trace -- python bench.py --config "$cfg" --steps 3 --no-cpu --no-fullscale \
            --no-fullscale-cifar10 --no-second --no-cifar10 --no-f32 --no-dropin
        line "$O/trace_$cfg.log" ;;
    pmc)
        OUT=$O/pmc bash tools/pmc.sh > "$O/pmc.log" 2>&1 || { tail -n 30 "$O/pmc.log"; exit 1; }
        python3 tools/pmc_r2.py "$O/pmc" "$O/net_pmc.json" > /dev/null || exit 1
        echo "== pmc -> $O/net_pmc.json" ;;
    pmc_flops)
        OUT=$O/pmc_flops bash tools/pmc_flops.sh > "$O/pmc_flops.log" 2>&1 || \
            { tail -n 30 "$O/pmc_flops.log"; exit 1; }
        grep -E "executed_flops_per_pair|lane_fill|executed_tflops" "$O/pmc_flops.log" ;;
    pmc_ta)
        PMC_CFGS="${PMC_CFGS:-mnist_paper_convnet_gp mnist_as_tf cifar10}" OUT=$O/pmc_ta \
            bash tools/pmc_ta.sh > "$O/pmc_ta.log" 2>&1 || { tail -n 30 "$O/pmc_ta.log"; exit 1; }
        tail -n 5 "$O/pmc_ta.log" ;;
    fullscale)
        step fullscale 900 python tools/fullscale.py ${FS_ARGS:-}
        tail -n 1 "$O/fullscale.log" ;;
    ab)
        if [ -n "${AB_TEST:-}" ]; then   # each variant's whole-network parity first
            for v in ${AB:-cur}; do
                [ "$v" = cur ] && continue
                CNNGP_LIB=$PWD/cnn-gp_amd/lib/ab/lib_$v.so step "abtest_$v" 600 python -u -m \
                    pytest tests/test_gpu_parity.py -x -q -k "netfuse or e2e or program" \
                    --timeout 300 --timeout-method thread
                tail -n 1 "$O/abtest_$v.log"
            done
        fi
        for rep in $(seq 1 "${AB_REPS:-2}"); do
            for v in ${AB:-cur}; do
                # NAME=VALUE: the current library with that environment variable set
                lib=$PWD/cnn-gp_amd/lib/libcnngp.so; envset=""; tag=$v
                case $v in
                cur) ;;
                *=*) envset=$v; tag=${v//[^A-Za-z0-9]/_} ;;
                *) lib=$PWD/cnn-gp_amd/lib/ab/lib_$v.so ;;
                esac
                env $envset CNNGP_LIB=$lib bash -c "$(declare -f step); O=$O; \
                    step ab_${tag}_$rep 300 python ${AB_TOOL:-tools/netbench.py} ${NB_ARGS:-}" || exit 1
                echo "-- $v (round $rep)"; grep -v amdgpu.ids "$O/ab_${tag}_$rep.log" | tail -n 8
            done
        done ;;
    envtest)
        # parity under an environment setting: ENVTEST="NAME=VALUE" PYTEST_ARGS="files -k expr"
        env ${ENVTEST} bash -c "$(declare -f step); O=$O; step envtest 900 python -u -m \
            pytest ${PYTEST_ARGS:-tests/test_gpu_parity.py} -x -q --timeout 300 \
            --timeout-method thread" || exit 1
        tail -n 1 "$O/envtest.log" ;;
    py:*)
        p=${s#py:}
        step "py_$(basename "$p" .py)" 600 python "$p" ${PY_ARGS:-}
        tail -n 30 "$O/py_$(basename "$p" .py).log" ;;
    *)
        echo "unknown step $s"; exit 2 ;;
    esac
done
echo "== done"
