#!/bin/bash
# One GPU-box session, run as:  gpurun -- 'bash tools/gpu.sh STEP [STEP ...]'
# Steps run in order, each under its own time limit; the first failing step ends the session.
#
#   smoke           __graft_entry__.smoke()
#   test            pytest ${TESTS:-tests -m gpu} ${TESTK:+-k $TESTK}          -> gpurun_out/pytest.log
#   bench           bench.py --steps 20 --warmup 5 $BENCH_ARGS                  -> gpurun_out/bench.log
#   ab              alternating bench runs of $VARIANTS (";"-separated "ENV=.. -- bench args"
#                   strings), $REPS rounds                                       -> gpurun_out/ab.log
#   prof            rocprofv3 --kernel-trace --stats of bench.py $BENCH_ARGS     -> gpurun_out/prof_$TAG
#   pmc             HBM-traffic / MFMA-busy counter passes of bench.py (tools/pmc_collect.py)
#   convbench       tools/convbench.py $CB_ARGS                                 -> gpurun_out/convbench.log
#   cbab            alternating convbench runs of $VARIANTS (";"-separated "ENV=.. -- convbench args"
#                   strings, e.g. "-- --lib face-vae_amd/csrc/build_ab/libfacevae_base.so;"), $REPS rounds
#   convpmc         SQ stall-anatomy counter passes over tools/convbench.py ($CB_ARGS)
#   c3pmc           SQ + FETCH/WRITE_SIZE counter passes over tools/conv3dbench.py ($C3_ARGS)
#   configs         bench lines of the other BASELINE configs on one GPU (512x512 B=8; B=64 bf16 / fp8)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
TAG=${TAG:-it}

line() { python tools/benchline.py < "$1"; }

step_smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -20 $O/smoke.log; return 1; }
  tail -1 $O/smoke.log
}

step_test() {
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests -m gpu} ${TESTK:+-k "$TESTK"} -x -v -s \
    --timeout ${PER_TEST_TIMEOUT:-300} --timeout-method thread > $O/pytest.log 2>&1
  local rc=$?
  echo "pytest exit $rc" >> $O/pytest.log
  grep -E "^(PASSED|FAILED)|passed|failed|deviation" $O/pytest.log | tail -${TEST_TAIL:-6}
  [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" $O/pytest.log | head -20; return 1; }
}

step_bench() {
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench.log 2>&1 \
    || { tail -20 $O/bench.log; return 1; }
  line $O/bench.log
}

step_ab() {
  : > $O/ab.log
  IFS=';' read -ra VS <<< "$VARIANTS"
  for i in $(seq 1 ${REPS:-3}); do
    for v in "${VS[@]}"; do
      local envs="${v%%--*}" args=""
      [[ "$v" == *--* ]] && args="${v#*--}"
      echo "== $v" >> $O/ab.log
      env FV_X=0 $envs timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 $args >> $O/ab.log 2>&1 \
        || { tail -20 $O/ab.log; return 1; }
    done
  done
  python tools/ab_summary.py $O/ab.log
}

step_prof() {
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 ${BENCH_ARGS:-} > $O/prof_$TAG.log 2>&1) \
    || { tail -20 $O/prof_$TAG.log; return 1; }
  tail -1 $O/prof_$TAG.log | cut -c1-200
}

step_pmc() {
  local B="$R/bench.py --steps 2 --warmup 1 --cpu-seconds 0 ${BENCH_ARGS:-}"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pmc_trace -o run -- \
    python3 $B > $O/pmc_trace.log 2>&1) || { echo "trace failed"; tail -5 $O/pmc_trace.log; return 1; }
  local i=0 c
  for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_p$i -o run -- \
      python3 $B > $O/pmc_p$i.log 2>&1) || { echo "pmc $c failed"; tail -5 $O/pmc_p$i.log; return 1; }
  done
  python tools/pmc_collect.py --trace $O/pmc_trace --pass $O/pmc_p1 --pass $O/pmc_p2 --pass $O/pmc_p3 > $O/pmc.json
}

step_convbench() {
  timeout -k 10 300 python tools/convbench.py ${CB_ARGS:-} > $O/convbench.log 2>&1 || { tail -20 $O/convbench.log; return 1; }
  grep -v amdgpu.ids $O/convbench.log
}

step_cbab() {
  : > $O/cbab.log
  IFS=';' read -ra VS <<< "$VARIANTS"
  for i in $(seq 1 ${REPS:-2}); do
    for v in "${VS[@]}"; do
      local envs="${v%%--*}" args=""
      [[ "$v" == *--* ]] && args="${v#*--}"
      echo "== $v" >> $O/cbab.log
      env FV_X=0 $envs timeout -k 10 200 python tools/convbench.py ${CB_ARGS:-} $args >> $O/cbab.log 2>&1 \
        || { tail -20 $O/cbab.log; return 1; }
    done
  done
  python tools/showbench.py < $O/cbab.log | head -150
}

step_convpmc() {
  local C="$R/tools/convbench.py --iters 5 ${CB_ARGS:---layers res --only fwd,wgrad}" i=0 c
  for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_WAVES"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/cpmc_p$i -o run -- \
      python3 $C > $O/cpmc_p$i.log 2>&1) || { echo "pmc pass $i failed"; tail -5 $O/cpmc_p$i.log; return 1; }
  done
  python tools/pmc_sq.py $O/cpmc_p1 $O/cpmc_p2 $O/cpmc_p3 | tee $O/convpmc.txt
}

step_c3pmc() {   # SQ + HBM counter passes over tools/conv3dbench.py ($C3_ARGS)
  local C="$R/tools/conv3dbench.py --iters 5 ${C3_ARGS:---batch 32}" i=0 c
  for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/c3pmc_p$i -o run -- \
      python3 $C > $O/c3pmc_p$i.log 2>&1) || { echo "pmc pass $i failed"; tail -5 $O/c3pmc_p$i.log; return 1; }
  done
  python tools/pmc_sq.py $O/c3pmc_p1 $O/c3pmc_p2 $O/c3pmc_p3 $O/c3pmc_p4 | tee $O/c3pmc.txt
}

step_configs() {
  local a
  for a in "--res 512 --batch 8" "--batch 64" "--batch 64 --dtype fp8"; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 $a > $O/bench_cfg.log 2>&1 \
      || { tail -20 $O/bench_cfg.log; return 1; }
    echo "[$a]"; line $O/bench_cfg.log
    cp $O/bench_cfg.log "$O/bench_$(echo $a | tr -d ' -').log"
  done
}

for s in "$@"; do
  echo "### $s"
  "step_$s" || { echo "step $s failed"; exit 1; }
done
