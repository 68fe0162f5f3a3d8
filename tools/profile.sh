#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then one PMC
# pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 50 --warmup 5 --no-cpu-baseline --no-wire --fresh-workers 0}
run() {  # name, limit, rocprof args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -n 3 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
run trace 400 --kernel-trace --stats
run pmc_fetch 400 --kernel-trace --pmc FETCH_SIZE
run pmc_write 400 --kernel-trace --pmc WRITE_SIZE
run pmc_sq 400 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
run pmc_sq2 400 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD
run pmc_tcc 400 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum
run pmc_wait 400 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
run pmc_lds 400 --kernel-trace --pmc SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_SALU
# summaries only (the raw traces exceed what gpurun copies back)
python tools/summarize_profile.py --src $OUT --tag ${TAG:-round2} --config ${CFG:-2} --envs ${ENVS:-4096} --out gpurun_out/psum || exit 1
rm -rf $OUT
exit 0
