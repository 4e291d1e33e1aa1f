set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARIANTS:-ring pool}; do
  export CNNGP_LIB=$PWD/cnn-gp_amd/lib/var/lib_$v.so
  timeout -k 10 200 python bench.py --config mnist_as_tf --no-cpu --no-probe > gpurun_out/ab_$v.json 2>/dev/null || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
