#!/bin/bash
# One entry point for the GPU-box runs (replaces the round-1 one-off scripts).
#
#   scripts/gpu.sh TASK [TASK ...]      e.g.  scripts/gpu.sh tests bench dp accuracy
#
# Every GPU step runs under its own `timeout -k 10`, output goes under
# gpurun_out/<task>/, and the script stops at the first failing step (no GPU
# work after a fault, abort or time limit).
#
# tasks:
#   build      rebuild every extension from source ON THE BOX (build_ext --force, both
#              libraries), so a session proves the pushed sources compile there
#   tests      pytest -m gpu (+ smoke)                    gpurun_out/tests/
#   bench      bench.py config 2, 20 steps, --verify      gpurun_out/bench/
#   configs    bench.py configs 3, 4 (fused + separate), 5
#   skew       bench.py --skew 2 and 3
#   dp         bench.py --gpus 2, 4 and 8 on this one GPU (gloo rehearsal of the spawn path)
#   accuracy   sweep-DP accuracy, 8 ranks x 10M matches over 1M players, sweeps 1,2,4,8
#   graph      micro-batches (eager vs HIP graph, scripts/bench_graph.py) + prepass alone
#   hop        quick executor A/B (serial chain + 10M window, local hand-off, timing build)
#   merge      sweep-merge message/decode kernels at P = 1M, 10M on one GPU
#   exactdp    exact DP (C2) rehearsal, 2/4 gloo ranks on one GPU, rounds + time per window
#   role       config 4 fused executor with dedicated aggregation waves (ANA_TELE_ROLE sweep)
#   slices     sweep-DP accuracy and 1-GPU step time vs slice size (fixed 80M-match history)
#   excl       prepass on its own CUs beside the executor on the rest (ANA_PREPASS_EXCLUSIVE sweep)
#   tele       config 4 telemetry placement (separate / fused / CU-masked overlap)
#   teleab     config 4 A/B of builds (AB_LIBS), optional tail-point sweep (TELEAB_TAIL_AT)
#   tail       prepass start point sweep for config 2 (ANA_PREPASS_AT, serial)
#   ab         in-call A/B of executor builds (AB_LIBS, scripts/ab_build.sh), interleaved rounds
#   micro      executor hop latency A/B (scripts/tune_rate.py: serial / uniform / skewed, timing build)
#   prof       rocprofv3 --kernel-trace --stats of config 2
#   pmc        rocprofv3 --pmc passes over the executor (10M-match window, tune_rate.py: one
#              process, no side-stream waits -- counter collection serialises dispatches, and a
#              stream wait on the executor's tail signal then never returns)
#   telepmc    rocprofv3 counters of the standalone telemetry aggregation
#   rerate     config 5 end to end: 1B matches / 10M players, checkpoint + kill + resume
#   worker     streaming worker on the device (ENGINE=native), memory + sqlite stores
#   workersql  the worker on the reflected SQLAlchemy store (columnar batch path), sqlite file
#   dpacc      sweep-DP accuracy table (ranks x merges per step) incl. per-participant records
#   dpcost     one-GPU DP step price: plain vs forced merges at k = 8 / 16
#   dpstep     forced-merge step price: record correction on / off, tail / serial placement, emulated N = 8
#   replicas   worker.py --replicas 1 / 2 / 4 on the box (shared broker + SQLite store)
#   dpconf     gloo rehearsals of config 3 (N = 4) and config 5 (N = 2)
#   rerate_dp  config-5-shaped re-rate over 2 gloo ranks on this GPU: checkpoint, kill, resume, bit-identity
#   project    one-GPU projection of the N = 2 / 4 / 8 DP step (emulated all-reduce, bus bandwidth sweep)
#   corrmicro  the record correction kernel alone + a kernel trace of the k = 8 DP step
#   gtest      a subset of the GPU tests (GTEST_K = pytest -k expression)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
PY=python3

run() {  # run NAME SECONDS CMD...: one bounded step, output to gpurun_out/NAME.log
  local name=$1 secs=$2; shift 2
  mkdir -p "$ROOT/gpurun_out/$(dirname "$name")"
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -3 "$ROOT/gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; exit $rc; fi
}

for task in "$@"; do
  case $task in
    build)  # CPU only: hipcc cross-compiles gfx950; the pushed .so files are replaced
      run build/build 900 $PY -m analyzer_amd.build_ext --force --jobs 16
      run build/build_diag 900 $PY -m analyzer_amd.build_ext --force --diag --jobs 16
      run build/import 120 $PY -c "from analyzer_amd.ops.native import native; native(); print('native ok')"
      ;;
    gtest)
      run gtest/pytest 600 $PY -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${GTEST_K}"
      ;;
    tests)
      run tests/pytest 900 $PY -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
      run tests/smoke 300 $PY -c "import __graft_entry__ as g; g.smoke()"
      ;;
    bench)
      run bench/config2 400 $PY bench.py --steps 20 --warmup 3 --check --verify
      ;;
    configs)
      run bench/config3 400 $PY bench.py --config 3 --steps 10 --warmup 2 --check
      run bench/config4_auto 400 $PY bench.py --config 4 --steps 10 --warmup 2
      run bench/config4_fused 400 $PY bench.py --config 4 --steps 10 --warmup 2 --telemetry-mode fused
      run bench/config4_separate 400 $PY bench.py --config 4 --steps 10 --warmup 2 --telemetry-mode separate
      run bench/config5 400 $PY bench.py --config 5 --steps 10 --warmup 2 --check
      ;;
    skew)
      run bench/skew2 600 $PY bench.py --skew 2 --steps 3 --warmup 1 --check
      run bench/skew3 900 $PY bench.py --skew 3 --steps 2 --warmup 1 --check
      ;;
    dp)
      run dp/gloo2 600 env ANA_DIST_BACKEND=gloo $PY bench.py --gpus 2 --steps 5 --warmup 2
      run dp/gloo4 900 env ANA_DIST_BACKEND=gloo $PY bench.py --gpus 4 --steps 3 --warmup 1
      run dp/gloo8 900 env ANA_DIST_BACKEND=gloo $PY bench.py --gpus 8 --steps 2 --warmup 1
      run dp/gloo2_sweeps2 600 env ANA_DIST_BACKEND=gloo $PY bench.py --gpus 2 --steps 3 --warmup 1 --sweeps 2
      ;;
    accuracy)
      run accuracy/dp8 900 $PY -m analyzer_amd.parallel.accuracy --device cuda --ranks 8 \
          --players 1e6 --matches-per-rank 1e7 --windows 1 --warm-windows 1 --sweeps 1,2,4,8
      run accuracy/dp4_skew 900 $PY -m analyzer_amd.parallel.accuracy --device cuda --ranks 4 \
          --players 2e4 --matches-per-rank 2e5 --windows 8 --warm-windows 1 --sweeps 1,2,3,4
      ;;
    idle)  # idle back-off and grid size sweep of the executor (10M window + serial chain)
      run idle/random 400 $PY scripts/tune_rate.py --pattern random --rounds 2 --idle=-1,2,8,16 --blocks 512,1024
      run idle/serial 300 $PY scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 --rounds 2 \
          --blocks 8 --idle=-1,2,8
      grep -h "^round 1" gpurun_out/idle/*.log | cut -c1-120
      ;;
    graph)  # worker-sized micro-batches: eager vs HIP-graph replay; schedule prepass alone
      run graph/microbatch 300 $PY scripts/bench_graph.py
      run graph/sched 300 $PY scripts/sched_time.py
      ;;
    hop)  # quick executor A/B: serial chain + 10M window, production + timing build
      run hop/serial 300 $PY scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 \
          --rounds 2 --blocks 8 --local 1 --diag 0,1
      run hop/random 300 $PY scripts/tune_rate.py --pattern random --rounds 3 --local 1 --diag 0,1
      grep -h "^round" gpurun_out/hop/*.log | cut -c1-420
      ;;
    ab)  # in-call A/B of executor builds: AB_LIBS="name:ab/name_C.so ..." ("cur:" = the tree's),
         # rounds interleaved so box drift hits every build alike (scripts/ab_build.sh)
      for r in 1 2 3; do
        for spec in ${AB_LIBS:-cur:}; do
          name=${spec%%:*}; lib=${spec#*:}
          ANA_NATIVE_LIB=$lib run ab/serial_${name}_$r 300 $PY scripts/tune_rate.py --pattern serial --players 1000 \
              --matches 20000 --rounds 1 --blocks 8 --local 1 --diag 0
          ANA_NATIVE_LIB=$lib run ab/random_${name}_$r 300 $PY scripts/tune_rate.py --pattern random --rounds 2 \
              --local 1 --diag 0
        done
      done
      for f in gpurun_out/ab/*.log; do
        echo "$f $(grep -h '^round' $f | sed -E 's/.*schedule +([0-9.]+) ms rate +([0-9.]+) ms.*/sched \1 rate \2 |/' | tr '\n' ' ')"
      done
      ;;
    merge)  # sweep-merge kernels (messages, decode) at 1M and 10M players, no collective
      run merge/kernels 300 $PY scripts/merge_micro.py --players 1e6,1e7
      ;;
    exactdp)  # exact DP rehearsal: 2 and 4 gloo ranks on this one GPU, 1M-match window
      run exactdp/r2 600 $PY scripts/exact_dp_rehearsal.py --ranks 2
      run exactdp/r4 600 $PY scripts/exact_dp_rehearsal.py --ranks 4
      ;;
    role)  # config 4 fused executor: dedicated aggregation waves (ANA_TELE_ROLE) vs idle-wave tiles vs separate
      run role/test 300 $PY -u -m pytest tests/test_engine_gpu.py -k fused_rate_telemetry -x -v --timeout 120 --timeout-method thread
      run role/separate 400 $PY bench.py --config 4 --steps 10 --warmup 2 --telemetry-mode separate
      for n in ${ROLES:-0 2 4 8 16}; do
        ANA_TELE_ROLE=$n run role/fused_role$n 400 $PY bench.py --config 4 --steps 10 --warmup 2 --telemetry-mode fused
      done
      ;;
    slices)  # sweep-DP accuracy vs slice size at a fixed 80M-match history (8 ranks, 1M players) + 1-GPU window time
      for w in 1 2 4 8; do
        mpr=$((10000000 / w))
        run slices/acc_w$w 600 $PY -m analyzer_amd.parallel.accuracy --device cuda --ranks 8 --players 1e6 \
            --matches-per-rank $mpr --windows $w --warm-windows 1 --sweeps 1,2
        run slices/bench_w$w 300 $PY bench.py --matches-per-gpu $mpr --steps $((20 * w)) --warmup 3
      done
      run slices/acc_fp16 600 $PY -m analyzer_amd.parallel.accuracy --device cuda --ranks 8 --players 1e6 \
          --matches-per-rank 10000000 --windows 1 --warm-windows 1 --sweeps 1 --comm-dtype fp16
      run slices/acc_bf16 600 $PY -m analyzer_amd.parallel.accuracy --device cuda --ranks 8 --players 1e6 \
          --matches-per-rank 10000000 --windows 1 --warm-windows 1 --sweeps 1 --comm-dtype bf16
      ;;
    excl)  # prepass of window i+1 on n CUs of its own while the executor rates window i on the others
      run excl/serial 400 $PY bench.py --steps 20 --warmup 3
      for n in ${EXCL_CUS:-32 48 64}; do
        ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=0 ANA_PREPASS_CUS=$n ANA_PREPASS_EXCLUSIVE=1 ANA_RATE_BLOCKS=$((2 * (256 - n))) \
          run excl/cus$n 400 $PY bench.py --steps 20 --warmup 3 --check
      done
      run excl/c3_default 400 $PY bench.py --config 3 --steps 10 --warmup 2
      for n in ${EXCL_CUS3:-48 64}; do
        ANA_PREPASS_AT=0 ANA_PREPASS_CUS=$n ANA_PREPASS_EXCLUSIVE=1 ANA_RATE_BLOCKS=$((2 * (256 - n))) \
          run excl/c3_cus$n 400 $PY bench.py --config 3 --steps 10 --warmup 2 --check
      done
      grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/excl/*.log
      ;;
    tele)  # config 4 telemetry placement: separate, fused, overlap on all / 16 / 32 / 64 CUs
      run tele/separate 400 $PY bench.py --config 4 --steps 10 --warmup 2 --telemetry-mode separate
      run tele/fused 400 $PY bench.py --config 4 --steps 10 --warmup 2 --telemetry-mode fused
      for n in ${TELE_CUS:-0 16 32 64}; do
        ANA_TELE_CUS=$n run tele/overlap_cus$n 400 $PY bench.py --config 4 --steps 10 --warmup 2 --telemetry-mode overlap
      done
      for f in gpurun_out/tele/*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
      ;;
    teleab)  # config 4 A/B of builds (AB_LIBS as for ab): bench step + the standalone aggregation, interleaved
      for r in $(seq ${TELEAB_ROUNDS:-3}); do
        for spec in ${AB_LIBS:-cur:}; do
          name=${spec%%:*}; lib=${spec#*:}
          ANA_NATIVE_LIB=$lib run teleab/bench_${name}_$r 300 $PY bench.py --config 4 --steps 10 --warmup 2
          [ "${TELEAB_KERNEL:-1}" = 0 ] || \
            ANA_NATIVE_LIB=$lib run teleab/kernel_${name}_$r 300 $PY scripts/tune_tele.py --variants impl1 --rounds 1
          for at in ${TELEAB_TAIL_AT:-}; do
            ANA_TELE_TAIL_AT=$at ANA_NATIVE_LIB=$lib run teleab/bench_${name}_at${at}_$r 300 $PY bench.py --config 4 \
                --steps 10 --warmup 2
          done
        done
      done
      for f in gpurun_out/teleab/bench_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done | sort
      ;;
    tail)  # where the next window's prepass starts (ANA_PREPASS_AT sweep, config 2; 0 = with the launch)
      for r in 1 2; do
        for at in ${TAIL_AT:-0.8 0.9}; do
          ANA_PREPASS_SERIAL=0 ANA_PREPASS_AT=$at run tail/config2_at${at}_$r 400 $PY bench.py --steps 20 --warmup 3
        done
        ANA_PREPASS_SERIAL=1 run tail/config2_serial_$r 400 $PY bench.py --steps 20 --warmup 3
      done
      for f in gpurun_out/tail/*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
      ;;
    micro)  # executor hop latency: serial chain, uniform window, skewed window (timing build A/B)
      run micro/serial 300 $PY scripts/tune_rate.py --pattern serial --players 1000 --matches 20000 \
          --rounds 2 --blocks ${MICRO_BLOCKS:-8,512} --local ${MICRO_LOCAL:-0,1} --diag 0,1
      run micro/random 300 $PY scripts/tune_rate.py --pattern random --rounds 2 --local ${MICRO_LOCAL:-0,1} --diag 0,1
      run micro/skew3 600 $PY scripts/tune_rate.py --pattern random --skew 3 --matches 2000000 --rounds 1 \
          --blocks ${MICRO_BLOCKS:-8,512} --local 1 --diag 0,1
      ;;
    prof)
      mkdir -p gpurun_out/prof
      (cd /tmp && run prof/config2 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof/config2" \
          -o run --output-format csv -- $PY "$ROOT/bench.py" --steps 5 --warmup 2 ${PROF_ARGS:-}) || exit $?
      $PY scripts/prof_summary.py gpurun_out/prof/config2/run_kernel_trace.csv | tee gpurun_out/prof/config2/summary.txt
      ;;
    pmc)
      # PMC_TAG / PMC_ARGS select the workload (default: the 10M-match bench window)
      tag=${PMC_TAG:-window}
      for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
                 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM" \
                 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT" \
                 "GRBM_GUI_ACTIVE GRBM_COUNT"; do
        name=$(echo $set | cut -d' ' -f1)
        (cd /tmp && run pmc/$tag/$name 120 rocprofv3 --pmc $set --kernel-trace --stats \
            -d "$ROOT/gpurun_out/pmc/$tag/$name" -o run --output-format csv -- $PY "$ROOT/scripts/tune_rate.py" \
            --rounds 1 ${PMC_ARGS:-}) || exit $?
        $PY scripts/pmc_kernel.py "gpurun_out/pmc/$tag/$name" rate_dataflow >> gpurun_out/pmc/$tag/executor.txt
      done
      cat gpurun_out/pmc/$tag/executor.txt
      ;;
    telepmc)  # counters of the standalone K8 aggregation (10M 3v3 window, ~400M events)
      for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
                 "FETCH_SIZE" "WRITE_SIZE"; do
        name=$(echo $set | cut -d' ' -f1)
        (cd /tmp && run telepmc/$name 120 rocprofv3 --pmc $set --kernel-trace --stats \
            -d "$ROOT/gpurun_out/telepmc/$name" -o run --output-format csv -- $PY "$ROOT/scripts/tele_once.py") || exit $?
        $PY scripts/pmc_kernel.py "gpurun_out/telepmc/$name" telemetry_kernel >> gpurun_out/telepmc/tele.txt
      done
      cat gpurun_out/telepmc/tele.txt
      ;;
    rerate)
      rm -rf /tmp/ck5
      rm -rf /tmp/ck5_full
      run rerate/full 900 $PY -m analyzer_amd.runtime.rerate --matches 1e9 --players 1e7 --window 1.6e7 \
          --checkpoint-dir /tmp/ck5_full --checkpoint-every 8 --digests
      # injected crash after 20 windows, then resume from the checkpoint of window 16
      mkdir -p gpurun_out/rerate
      echo "== rerate/kill"
      timeout -k 10 600 $PY -m analyzer_amd.runtime.rerate --matches 1e9 --players 1e7 --window 1.6e7 \
          --checkpoint-dir /tmp/ck5 --checkpoint-every 8 --fault-kill-after 20 > gpurun_out/rerate/kill.log 2>&1
      rc=$?; tail -2 gpurun_out/rerate/kill.log
      if [ $rc -ne 17 ]; then echo "!! expected exit 17 from the injected fault, got $rc"; exit 1; fi
      run rerate/resume 900 $PY -m analyzer_amd.runtime.rerate --matches 1e9 --players 1e7 --window 1.6e7 \
          --checkpoint-dir /tmp/ck5 --checkpoint-every 8 --digests
      $PY - <<'EOF'
import json
full = json.loads(open("gpurun_out/rerate/full.log").read().strip().splitlines()[-1])
res = json.loads(open("gpurun_out/rerate/resume.log").read().strip().splitlines()[-1])
g0 = int(res["resumed_from_window"])
same = all(full["window_digests"][g] == d for g, d in res["window_digests"].items())
print("resumed from window", g0, "| roster bit-identical:", full["roster_sha256"] == res["roster_sha256"],
      "| re-rated windows' records identical:", same, "| participant records (full run):",
      full["participant_records"])
EOF
      run rerate/host_egress 900 $PY -m analyzer_amd.runtime.rerate --matches 2e8 --players 1e7 \
          --window 1.6e7 --records host
      ;;
    worker)  # the streaming worker, BATCHSIZE=500: columnar / object / SQLite stores, native vs python
      run worker/columnar_native 600 env DATABASE_URI=columnar:// ENGINE=native BATCHSIZE=500 \
          IDLE_TIMEOUT=0.01 $PY worker.py --synthetic 200000
      run worker/columnar_native_telemetry 600 env DATABASE_URI=columnar:// ENGINE=native DOTELEMETRY=true \
          BATCHSIZE=500 IDLE_TIMEOUT=0.01 $PY worker.py --synthetic 200000
      run worker/memory_native 600 env ENGINE=native BATCHSIZE=500 IDLE_TIMEOUT=0.01 $PY worker.py --synthetic 50000
      run worker/memory_python 600 env ENGINE=python BATCHSIZE=500 IDLE_TIMEOUT=0.01 $PY worker.py --synthetic 20000
      run worker/sqlite_native 600 env DATABASE_URI=sqlite:////tmp/wn.db ENGINE=native BATCHSIZE=500 \
          IDLE_TIMEOUT=0.01 $PY worker.py --synthetic 50000
      run worker/sqlite_python 600 env DATABASE_URI=sqlite:////tmp/wp.db ENGINE=python BATCHSIZE=500 \
          IDLE_TIMEOUT=0.01 $PY worker.py --synthetic 20000
      # per-stage profiles (scripts/worker_profile.py): columnar serial x2 / pipelined, SQLite, SQLAlchemy
      run worker/profiles 900 bash scripts/worker_stores.sh
      ;;
    dpacc)  # sweep-DP accuracy incl. the per-participant records, (ranks x merges per step), 3v3 bench shape
      run dpacc/table 900 $PY scripts/merges_vs_ranks.py ${DPACC_PAIRS:-2x2,4x4,4x8,8x8,8x16}
      cat gpurun_out/dpacc/table.log
      ;;
    dpcost)  # one-GPU price of the DP step: plain vs forced merges at k = 8 / 16 (interleaved rounds)
      for r in 1 2; do
        run dpcost/plain_$r 300 $PY bench.py --steps 10 --warmup 2
        for k in ${DPCOST_K:-8 16}; do
          run dpcost/k${k}_$r 300 $PY bench.py --steps 10 --warmup 2 --force-merge --merges-per-step $k
        done
      done
      for f in gpurun_out/dpcost/*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
      ;;
    dpstep)  # one-GPU DP step price: plain vs forced merges (DPSTEP_K); record correction on (default) / off;
             # serial placement; N = 8 projected with the all-reduce stand-in (8 ranks, 300 GB/s); interleaved rounds
      for r in 1 2; do
        run dpstep/plain_$r 300 $PY bench.py --steps 10 --warmup 2
        for k in ${DPSTEP_K:-8 16}; do
          A="--steps 10 --warmup 2 --force-merge --merges-per-step $k"
          run dpstep/k${k}_window_$r 300 $PY bench.py $A
          ANA_DP_CORRECT_RECORDS=0 run dpstep/k${k}_window_nocorr_$r 300 $PY bench.py $A
          ANA_PREPASS_SERIAL=1 run dpstep/k${k}_window_serial_$r 300 $PY bench.py $A
          run dpstep/k${k}_emu8_$r 300 $PY bench.py $A --emulate-allreduce 8:300
        done
      done
      for f in gpurun_out/dpstep/*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
      ;;
    replicas)  # worker scale-out on the box: 1 / 2 / 4 worker processes on one queue (tcp:// broker) over one
               # SQLite store file, ENGINE=native, 40k synthetic matches
      for n in 1 2 4; do
        rm -f /tmp/rep$n.db*
        ENGINE=native DATABASE_URI=sqlite:////tmp/rep$n.db run replicas/n$n 600 $PY worker.py --synthetic 40000 \
            --replicas $n
      done
      grep -h -o '"matches_per_s": [0-9.]*' gpurun_out/replicas/*.log
      ;;
    rerate_dp)  # P4 time-axis sharding end to end: 2 gloo ranks sharing this GPU (10M players, 2 x 16M matches per
                # global window, fp16 merges), checkpoint every 2 windows, kill after 5, resume, compare with a full run
      mkdir -p gpurun_out/rerate_dp
      rm -rf /tmp/ckdp /tmp/ckdp_full
      RDP="$PY -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
          -m analyzer_amd.runtime.rerate --matches 2.56e8 --players 1e7 --window 1.6e7 --checkpoint-every 2 --digests"
      ANA_DIST_BACKEND=gloo ANA_RATE_BLOCKS=256 run rerate_dp/full 900 $RDP --checkpoint-dir /tmp/ckdp_full
      echo "== rerate_dp/kill"
      ANA_DIST_BACKEND=gloo ANA_RATE_BLOCKS=256 timeout -k 10 900 $RDP --checkpoint-dir /tmp/ckdp --fault-kill-after 5 \
          > gpurun_out/rerate_dp/kill.log 2>&1
      rc=$?; tail -2 gpurun_out/rerate_dp/kill.log
      if [ $rc -eq 0 ]; then echo "!! expected a failure exit from the injected fault"; exit 1; fi
      ANA_DIST_BACKEND=gloo ANA_RATE_BLOCKS=256 run rerate_dp/resume 900 $RDP --checkpoint-dir /tmp/ckdp
      $PY - <<'EOF2'
import json
def last(p):
    return json.loads([l for l in open(p).read().splitlines() if l.startswith("{")][-1])
full, res = last("gpurun_out/rerate_dp/full.log"), last("gpurun_out/rerate_dp/resume.log")
same = all(full["window_digests"][g] == d for g, d in res["window_digests"].items())
print("2 ranks | resumed from window", int(res["resumed_from_window"]), "| roster bit-identical:",
      full["roster_sha256"] == res["roster_sha256"], "| re-rated windows' records identical:", same,
      "| full run %.2f s, %d windows" % (full["seconds"], full["windows"]))
EOF2
      ;;
    dpconf)  # gloo rehearsals of the other DP configs: 5v5 (config 3, k = 2N) and the 10M-player re-rate (config 5)
      run dpconf/c3_gloo4 900 env ANA_DIST_BACKEND=gloo $PY bench.py --config 3 --gpus 4 --steps 1 --warmup 1
      run dpconf/c5_gloo2 900 env ANA_DIST_BACKEND=gloo $PY bench.py --config 5 --gpus 2 --steps 1 --warmup 1
      ;;
    project)  # N-GPU step projection on one GPU: k = N forced merges with the all-reduce stand-in
              # (N ranks, BW GB/s bus bandwidth), N = 2 / 4 / 8 at 300 GB/s, N = 8 at 150 / 600 GB/s
      for r in 1 2; do
        run project/plain_$r 300 $PY bench.py --steps 10 --warmup 2
        for nb in 2:300 4:300 8:300 8:150 8:600; do
          n=${nb%%:*}
          run project/emu${nb/:/_}_$r 300 $PY bench.py --steps 10 --warmup 2 --force-merge --merges-per-step $n \
              --emulate-allreduce $nb
        done
      done
      for f in gpurun_out/project/*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
      ;;
    corrmicro)  # the record correction alone (scripts/correct_micro.py) + kernel trace of the forced k = 8 step
      run corrmicro/micro 300 $PY scripts/correct_micro.py
      run corrmicro/micro_10M 300 $PY scripts/correct_micro.py --matches 10e6
      run corrmicro/trace 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/corrmicro/prof" -o run \
          -- $PY bench.py --steps 4 --warmup 1 --force-merge --merges-per-step 8
      find gpurun_out/corrmicro/prof -name '*kernel_stats.csv' -exec head -25 {} \;
      ;;
    workersql)  # the streaming worker on the reflected SQLAlchemy store (sqlite file), native engine
      rm -f /tmp/wsa*.db*
      run workersql/sqla_native 600 $PY scripts/worker_profile.py --synthetic 100000 --cprofile 0 \
          --store "sqlalchemy+sqlite:////tmp/wsa1.db" --engine native
      RESIDENT=true run workersql/sqla_native_resident 600 $PY scripts/worker_profile.py --synthetic 100000 \
          --cprofile 0 --store "sqlalchemy+sqlite:////tmp/wsa2.db" --engine native
      run workersql/sqlite_native 600 $PY scripts/worker_profile.py --synthetic 100000 --cprofile 0 \
          --store "sqlite:////tmp/wsa3.db" --engine native
      grep -h -o '"matches_per_s": [0-9.]*' gpurun_out/workersql/*.log
      ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
