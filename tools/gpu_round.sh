#!/bin/bash
# GPU-box measurement script (one gpurun call).  Steps run in the order given; each GPU step
# has its own time limit and the chain stops at the first failure.
#   /usr/local/graft/bin/gpurun --timeout 1100 -- bash tools/gpu_round.sh <tag> <step>...
# steps:
#   tests[=filter]  pytest -m gpu (optionally -k filter)      smoke   __graft_entry__.smoke()
#   bench           headline bench.py (20 steps)              configs every BASELINE.json config
#   prof            rocprofv3 --kernel-trace --stats of the headline (10 steps)
#   profcfg=CFG     the same for another bench config (e.g. arcface)
#   profenv=V=X[:T] the headline profile with environment V=X (output prof_T)
#   profsmall       the same for the batch-32 HIP-graph step (200 replays)
#   pmcconv=S:CFGS  PMC passes (SQ / TCC hit-miss / FETCH_SIZE) over forward convs of shapes S under configs CFGS
#   graph1024       headline batch eager vs HIP graph, interleaved twice
#   ddpab           batch-32 graph: no DDP vs world-1 bucket engine variants (side stream, same stream, 100 MB buckets)
#   profddp         the same for the world-1 RCCL bucket-engine batch-32 HIP-graph step
#   graphs          HIP-graph batch 32 / 128 twice, then the headline batch
#   pmc             three PMC passes (SQ: MFMA busy / LDS conflicts / waits; FETCH_SIZE; WRITE_SIZE)
#   gloo2           bench.py --gpus 2 over gloo on this one GPU (self-launched ranks)
#   stock           stock PyTorch-ROCm ResNet-50 step (MIOpen / hipBLASLt) at batch 256
#   stock1024       the same at batch 1024 (the headline batch)
#   stockfp32       the same in fp32 (the reference's own precision), batch 256
#   sweep           headline batch sweep 128..2048
#   convbench       per-shape conv fwd/dgrad/wgrad timings vs the roofline (R50 shapes, b1024)
#   convbench32     the same at batch 32 (the reference's per-process batch)
#   benchab=CFG     headline bench default vs DCP_TUNE=CFG, interleaved twice
#   cfgab=CFG:A|B   bench.py --config CFG under DCP_TUNE=A vs DCP_TUNE=B (both disable the autotuner alike), twice
#   benchenv=V=X    headline bench default vs with environment V=X, interleaved twice
#   blas            torch.mm (hipBLASLt) on the R50 1x1 stride-1 GEMM shapes, b1024 (library yardstick)
#   small           the reference's per-process batches: b32 / b128, eager and HIP-graph replay
#   smallenv=V=X    b32 graph / b128 eager, default vs with environment V=X
#   large           ResNet-101 at per-GPU batch 2048 / 3072 (288 GB sizing, >2^32-element tensors)
#   gconvab=CFGS    ResNeXt-50 grouped convs under each g_tune config (",gconv_spw=1" = default vs one super-group)
#   convab=CFGS     tools/conv_bench.py --cfgs CFGS at b1024 (in-process interleaved A/B of g_tune configs)
#   loop            main.py's training loop vs bench.py at batch 32 (eager, HIP graph) and 128
#   ddp1            world-1 RCCL through the bucket engine (--force-ddp): b32 graph / eager, b1024 (+ SyncBN phase,
#                   comm telemetry), bf16 buckets
set -e
set -o pipefail
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
prof_env() { cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; }
for step in "$@"; do
  case $step in
    tests*)
      k=${step#tests}; k=${k#=}
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${k:+-k "$k"} \
        > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
      tail -2 $O/gpu_tests.log ;;
    probe)
      # world-1 RCCL DDP step with the collective probe in its JSON (comm_probe)
      timeout -k 10 300 python -u bench.py --force-ddp --steps 20 --warmup 5 > $O/ddp1_probe.log 2>&1
      tail -1 $O/ddp1_probe.log | grep -o '"comm_probe": {[^}]*}[^}]*}[^}]*}' ;;
    ddp1)
      timeout -k 10 300 python -u bench.py --force-ddp --batch 32 --graph --steps 100 --warmup 5 > $O/ddp1_b32g.log 2>&1
      tail -1 $O/ddp1_b32g.log
      timeout -k 10 300 python -u bench.py --force-ddp --batch 32 --steps 100 --warmup 5 > $O/ddp1_b32.log 2>&1
      tail -1 $O/ddp1_b32.log
      timeout -k 10 300 python -u bench.py --force-ddp --steps 20 --warmup 5 > $O/ddp1_b1024.log 2>&1
      tail -1 $O/ddp1_b1024.log
      timeout -k 10 300 python -u bench.py --force-ddp --batch 128 --grad-comm bf16 --steps 30 --warmup 5 > $O/ddp1_b128bf16.log 2>&1
      tail -1 $O/ddp1_b128bf16.log ;;
    refcfg)
      # the reference's own configurations (BASELINE/main.py:29-30,148; ARCFACE/arc_main.py:38,69-73,
      # arc_train_hpc.sh:3): small per-GPU batches, HIP graph and eager, local BN and world-1 RCCL SyncBN
      run_ref() {  # tag, bench args...
        local t=$1; shift
        timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 "$@" > $O/ref_$t.log 2>&1
        # (the JSON line is the last one starting with "{": a world-1 DDP run may print after it)
        echo "$t $(grep '^{' $O/ref_$t.log | tail -1 | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("syncbn_value"), r.get("syncbn_ms_per_step"))')"
      }
      run_ref tresnet_b16_graph --config tresnet --batch 16 --graph
      run_ref tresnet_b16_eager --config tresnet --batch 16 --eager
      run_ref tresnet_b16_ddp1_graph --config tresnet --batch 16 --force-ddp --graph
      run_ref tresnet_b16_ddp1_eager --config tresnet --batch 16 --force-ddp --eager
      for b in 16 32 64; do
        run_ref r50_b${b}_graph --batch $b --graph
        run_ref r50_b${b}_eager --batch $b --eager
        run_ref r50_b${b}_ddp1_graph --batch $b --force-ddp --graph
      done
      for b in 32 64; do
        run_ref arc256_b${b}_graph --config arcface --image-size 256 --batch $b --graph
        run_ref arc256_b${b}_eager --config arcface --image-size 256 --batch $b --eager
        run_ref arc256_b${b}_ddp1_graph --config arcface --image-size 256 --batch $b --force-ddp --graph
      done ;;
    gconvab=*)
      # gconvab=CFGS -- ResNeXt-50 grouped convs (fwd+stats / dgrad+BN / wgrad) under each g_tune config, b1024
      c=${step#gconvab=}
      timeout -k 10 400 python -u tools/conv_bench.py --grouped --batch 1024 --iters 10 --no-miopen --cfgs "$c" \
        > $O/gconvab.log 2>&1
      tail -4 $O/gconvab.log ;;
    convabs=*)
      # convabs=IDX,IDX:CFGS -- the same A/B on a subset of the R50 shapes (conv_bench.py R50 indices)
      v=${step#convabs=}; only=${v%%:*}; c=${v#*:}
      timeout -k 10 900 python -u tools/conv_bench.py --batch 1024 --iters 10 --only "$only" --cfgs "$c" \
        > $O/convabs.log 2>&1
      tail -3 $O/convabs.log ;;
    convab=*)
      c=${step#convab=}
      timeout -k 10 900 python -u tools/conv_bench.py --batch 1024 --iters 10 --only 1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22 --cfgs "$c" \
        > $O/convab.log 2>&1
      tail -3 $O/convab.log ;;
    loop)
      for g in "" "--graph"; do
        timeout -k 10 400 python -u tools/loop_vs_bench.py --batch 32 $g > $O/loop32$g.log 2>&1
        tail -1 $O/loop32$g.log
      done
      timeout -k 10 400 python -u tools/loop_vs_bench.py --batch 128 --steps 120 --log-interval 20 --bench-steps 40 \
        > $O/loop128.log 2>&1
      tail -1 $O/loop128.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
      tail -1 $O/bench.log ;;
    configs)
      for c in r50 arcface resnext r101 tresnet; do
        timeout -k 10 240 python -u bench.py --config $c --steps 20 --warmup 5 > $O/bench_$c.log 2>&1
        tail -1 $O/bench_$c.log
      done ;;
    gloo2)
      DCP_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --batch 256 --steps 5 --warmup 2 \
        > $O/bench_gloo2.log 2>&1
      tail -1 $O/bench_gloo2.log ;;
    prof)
      prof_env
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 30 --warmup 3 \
        > $O/prof.log 2>&1
      echo prof done ;;
    profenv=*)
      # profenv=V=X[:tag] -- the headline profile with environment V=X (kernel-level view of an A/B)
      a=${step#profenv=}; kv=${a%%:*}; tg=${a#*:}; [ "$tg" = "$a" ] && tg=env
      prof_env
      export "$kv"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$tg -o run -- python3 -u bench.py --steps 30 --warmup 3 \
        > $O/prof_$tg.log 2>&1
      unset "${kv%%=*}"
      echo prof $tg done ;;
    profcfg=*)
      # rocprofv3 kernel stats of another BASELINE config, e.g. profcfg=arcface
      c=${step#profcfg=}
      prof_env
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run -- python3 -u bench.py --config $c --steps 8 --warmup 2 \
        > $O/prof_$c.log 2>&1
      echo prof $c done ;;
    profsmall*)
      # profsmall[=ARGS]: kernel statistics + one-step timeline of a small-batch HIP-graph step after
      # autotuning (tuning cache replayed, last 100 replays counted): default R50 batch 32;
      # e.g. profsmall="--config tresnet --batch 16 --force-ddp --syncbn"
      args=${step#profsmall}; args=${args#=}; [ -z "$args" ] && args="--batch 32"
      tg=$(echo "$args" | tr -c 'a-z0-9' '_' | sed 's/__*/_/g; s/^_//; s/_$//')
      prof_env
      export DCP_TUNE_CACHE=$PWD/$O/profsmall_${tg}_tune.txt
      rm -f $DCP_TUNE_CACHE
      timeout -k 10 300 python3 -u bench.py $args --graph --steps 5 --warmup 5 > $O/profsmall_${tg}_tune.log 2>&1
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profsmall_$tg -o run -- python3 -u bench.py $args --graph --steps 100 --warmup 5 \
        > $O/profsmall_$tg.log 2>&1
      unset DCP_TUNE_CACHE
      python3 tools/rocpd_summary.py $O/profsmall_$tg/run_results.db --last-steps 100 --top 60 > $O/profsmall_${tg}_summary.txt 2>&1 || true
      python3 tools/step_timeline.py $O/profsmall_$tg/run_results.db > $O/profsmall_${tg}_step.txt 2>&1 || true
      tail -1 $O/profsmall_$tg.log; head -1 $O/profsmall_${tg}_summary.txt; tail -1 $O/profsmall_${tg}_step.txt ;;
    profddp)
      # rocprofv3 kernel statistics of the world-1 RCCL bucket-engine batch-32 HIP-graph step
      prof_env
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ddp -o run -- python3 -u bench.py --force-ddp --batch 32 --graph --steps 200 --warmup 5 --no-syncbn-phase --telemetry-steps 0 \
        > $O/prof_ddp.log 2>&1
      echo prof ddp done ;;
    ddpab)
      # batch-32 HIP-graph step: no DDP, world-1 bucket engine (default / compute-stream buckets /
      # one 100 MB bucket), interleaved twice
      for r in 1 2; do
        timeout -k 10 240 python -u bench.py --batch 32 --graph --steps 100 --warmup 5 > $O/ddpab_plain_$r.log 2>&1
        echo "plain: $(grep -o '"ms_per_step": [0-9.]*' $O/ddpab_plain_$r.log)"
        timeout -k 10 240 python -u bench.py --force-ddp --no-syncbn-phase --telemetry-steps 0 --batch 32 --graph --steps 100 --warmup 5 > $O/ddpab_ddp_$r.log 2>&1
        echo "ddp: $(grep -o '"ms_per_step": [0-9.]*' $O/ddpab_ddp_$r.log)"
        DCP_COMM_STREAM=0 timeout -k 10 240 python -u bench.py --force-ddp --no-syncbn-phase --telemetry-steps 0 --batch 32 --graph --steps 100 --warmup 5 > $O/ddpab_same_$r.log 2>&1
        echo "ddp same stream: $(grep -o '"ms_per_step": [0-9.]*' $O/ddpab_same_$r.log)"
        timeout -k 10 240 python -u bench.py --force-ddp --no-syncbn-phase --telemetry-steps 0 --bucket-cap-mb 100 --batch 32 --graph --steps 100 --warmup 5 > $O/ddpab_big_$r.log 2>&1
        echo "ddp 100MB buckets: $(grep -o '"ms_per_step": [0-9.]*' $O/ddpab_big_$r.log)"
      done ;;
    pmcconv=*)
      # PMC passes over forward convs of chosen shapes under chosen configs, e.g.
      # pmcconv=13,16:26=0,26=1 (tools/pmc_conv.py; kernels told apart by name)
      a=${step#pmcconv=}; shp=${a%%:*}; cf=${a#*:}
      prof_env
      export DCP_AUTOTUNE=0
      timeout -s KILL 60 rocprofv3 -L > $O/pmc_counters_avail.txt 2>&1 || true
      P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $O/pmcc1 -o run -- python3 -u tools/pmc_conv.py --only "$shp" --cfgs "$cf" > $O/pmcc1.log 2>&1
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/pmcc2 -o run -- python3 -u tools/pmc_conv.py --only "$shp" --cfgs "$cf" > $O/pmcc2.log 2>&1
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/pmcc3 -o run -- python3 -u tools/pmc_conv.py --only "$shp" --cfgs "$cf" > $O/pmcc3.log 2>&1
      echo pmcconv done ;;
    pmc6=*)
      # pmc6=SHAPES -- counter passes over the kernels the step runs for those R50 shapes (autotuned
      # choice; tools/pmc_r6.py, tools/pmc_r6_report.py): fwd / dgrad / wgrad, tuning dispatches excluded
      shp=${step#pmc6=}
      prof_env
      timeout -s KILL 60 rocprofv3 -L > $O/pmc_counters_avail.txt 2>&1 || true
      have() { local out=""; for c in "$@"; do grep -qw "$c" $O/pmc_counters_avail.txt && out="$out $c"; done; echo $out; }
      P1=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY)
      P2=$(have TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum)
      P3=$(have SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES)
      echo "P1=$P1 | P2=$P2 | P3=$P3"
      # one tuning run first: every counter pass then replays the same per-shape choices (a tuning
      # cache), so the passes count the same kernels (round-6 s1: independent tuning picked different
      # kernels in different passes for 5 of 36 blocks)
      export DCP_TUNE_CACHE=$PWD/$O/pmc6_tune.txt
      rm -f $DCP_TUNE_CACHE
      timeout -k 10 300 python3 -u tools/pmc_r6.py --only "$shp" --iters 1 > $O/pmc6_tune.log 2>&1
      i=0
      for P in "$P1 GRBM_GUI_ACTIVE" "$P2 GRBM_GUI_ACTIVE" "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE" "$P3 GRBM_GUI_ACTIVE"; do
        i=$((i+1))
        timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/pmc6/p$i -o run -- python3 -u tools/pmc_r6.py --only "$shp" > $O/pmc6_p$i.log 2>&1
        echo "pass $i done"
      done
      unset DCP_TUNE_CACHE
      python3 tools/pmc_r6_report.py $O/pmc6 --log $O/pmc6_p1.log > $O/pmc6_report.txt 2>&1 || true
      echo pmc6 done ;;
    profclean)
      # kernel statistics of the headline step AFTER autotuning: only the last 20 graph-replayed steps
      prof_env
      # tune in a first process (cache), profile a second that replays the choices: no tuning dispatches
      export DCP_TUNE_CACHE=$PWD/$O/profc_tune.txt
      rm -f $DCP_TUNE_CACHE
      timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 3 > $O/profc_tune.log 2>&1
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profc -o run -- python3 -u bench.py --steps 20 --warmup 5 \
        > $O/profc.log 2>&1
      unset DCP_TUNE_CACHE
      db=$O/profc/run_results.db
      python3 tools/rocpd_summary.py "$db" --last-steps 20 --top 60 > $O/profc_summary.txt 2>&1 || true
      python3 tools/step_timeline.py "$db" > $O/profc_step.txt 2>&1 || true
      tail -1 $O/profc.log; head -2 $O/profc_summary.txt; tail -1 $O/profc_step.txt ;;
    graph1024)
      # headline batch: eager vs HIP-graph replay, interleaved twice
      for r in 1 2; do
        timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --eager > $O/g1024_eager_$r.log 2>&1
        echo "eager: $(grep -o '"value": [0-9.]*' $O/g1024_eager_$r.log)"
        timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --graph > $O/g1024_graph_$r.log 2>&1
        echo "graph: $(grep -o '"value": [0-9.]*' $O/g1024_graph_$r.log)"
      done ;;
    graphs)
      # HIP-graph batch 32 / 128 (x2) and the headline batch
      for r in 1 2; do
        timeout -k 10 240 python -u bench.py --batch 32 --graph --steps 50 --warmup 5 > $O/g32_$r.log 2>&1
        echo "b32 graph $(grep -o '"value": [0-9.]*' $O/g32_$r.log)"
        timeout -k 10 240 python -u bench.py --batch 128 --graph --steps 30 --warmup 5 > $O/g128_$r.log 2>&1
        echo "b128 graph $(grep -o '"value": [0-9.]*' $O/g128_$r.log)"
      done
      timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > $O/b1024.log 2>&1
      echo "b1024 $(grep -o '"value": [0-9.]*' $O/b1024.log)" ;;
    pmc)
      prof_env
      export DCP_AUTOTUNE=0  # the heuristic's kernels: no tuning dispatches inside the counted steps
      PASS1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
      timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $PASS1 --output-format csv -d $O/pmc1 -o run -- python3 -u bench.py --steps 2 --warmup 1 > $O/pmc1.log 2>&1
      timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -o run -- python3 -u bench.py --steps 2 --warmup 1 > $O/pmc2.log 2>&1
      timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc3 -o run -- python3 -u bench.py --steps 2 --warmup 1 > $O/pmc3.log 2>&1
      echo pmc done ;;
    stock)
      timeout -k 10 600 python -u tools/bench_torch_reference.py --batch 256 --warmup 3 > $O/stock_r50_b256.log 2>&1
      tail -1 $O/stock_r50_b256.log ;;
    stock1024)
      timeout -k 10 600 python -u tools/bench_torch_reference.py --batch 1024 --warmup 3 > $O/stock_r50_b1024.log 2>&1
      tail -1 $O/stock_r50_b1024.log ;;
    stockfp32)
      timeout -k 10 600 python -u tools/bench_torch_reference.py --batch 256 --warmup 3 --fp32 > $O/stock_r50_b256_fp32.log 2>&1
      tail -1 $O/stock_r50_b256_fp32.log ;;
    sweep)
      for b in 128 256 512 1024 2048; do
        timeout -k 10 240 python -u bench.py --batch $b --steps 10 --warmup 3 > $O/sweep_b$b.log 2>&1
        tail -1 $O/sweep_b$b.log
      done ;;
    small)
      for b in 32 128; do
        timeout -k 10 240 python -u bench.py --batch $b --steps 30 --warmup 5 --eager > $O/small_b$b.log 2>&1
        tail -1 $O/small_b$b.log | grep -o '"value": [0-9.]*'
        timeout -k 10 240 python -u bench.py --batch $b --steps 30 --warmup 5 --graph > $O/small_b${b}_graph.log 2>&1
        tail -1 $O/small_b${b}_graph.log | grep -o '"value": [0-9.]*'
      done ;;
    smallenv=*)
      # b32 HIP-graph and b128 eager, default vs with an environment assignment
      c=${step#smallenv=}
      for args in "--batch 32 --graph" "--batch 128 --eager"; do
        tag=$(echo "$args" | tr -d ' -')
        timeout -k 10 240 python -u bench.py $args --steps 30 --warmup 5 > $O/smallenv_${tag}_default.log 2>&1
        echo "$args default: $(grep -o '"value": [0-9.]*' $O/smallenv_${tag}_default.log)"
        env "$c" timeout -k 10 240 python -u bench.py $args --steps 30 --warmup 5 > $O/smallenv_${tag}_set.log 2>&1
        echo "$args $c: $(grep -o '"value": [0-9.]*' $O/smallenv_${tag}_set.log)"
      done ;;
    large)
      for b in 2048 3072; do
        timeout -k 10 400 python -u bench.py --config r101 --batch $b --steps 5 --warmup 2 > $O/r101_b$b.log 2>&1
        tail -1 $O/r101_b$b.log
      done ;;
    convbench)
      timeout -k 10 400 python -u tools/conv_bench.py --batch 1024 --iters 10 --no-miopen > $O/conv_bench_b1024.txt 2>&1
      tail -3 $O/conv_bench_b1024.txt ;;
    convbench32)
      timeout -k 10 400 python -u tools/conv_bench.py --batch 32 --iters 50 --no-miopen > $O/conv_bench_b32.txt 2>&1
      tail -3 $O/conv_bench_b32.txt ;;
    ab=*)
      # per-shape in-process A/B of g_tune configs, e.g. ab=24=2,24=1,24=3
      c=${step#ab=}
      timeout -k 10 600 python -u tools/conv_bench.py --batch 1024 --iters 10 --no-miopen --cfgs "$c" \
        > $O/conv_ab_$(echo "$c" | tr ',;=' '_._').txt 2>&1
      tail -2 $O/conv_ab_*.txt ;;
    benchab=*)
      # headline bench, default vs DCP_TUNE=<cfg>, interleaved twice (same box, back to back)
      c=${step#benchab=}
      for r in 1 2; do
        timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/benchab_default_$r.log 2>&1
        echo "default: $(grep -o '"value": [0-9.]*' $O/benchab_default_$r.log)"
        DCP_TUNE="$c" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/benchab_tuned_$r.log 2>&1
        echo "DCP_TUNE=$c: $(grep -o '"value": [0-9.]*' $O/benchab_tuned_$r.log)"
      done ;;
    cfgab=*)
      # cfgab=CONFIG:A|B -- bench.py --config CONFIG under DCP_TUNE=A vs DCP_TUNE=B, interleaved twice
      v=${step#cfgab=}; cfg=${v%%:*}; ab=${v#*:}; A=${ab%%|*}; B=${ab#*|}
      for r in 1 2; do
        DCP_TUNE="$A" timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 5 > $O/cfgab_a_$r.log 2>&1
        echo "$cfg DCP_TUNE=$A: $(grep -o '"value": [0-9.]*' $O/cfgab_a_$r.log)"
        DCP_TUNE="$B" timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 5 > $O/cfgab_b_$r.log 2>&1
        echo "$cfg DCP_TUNE=$B: $(grep -o '"value": [0-9.]*' $O/cfgab_b_$r.log)"
      done ;;
    benchenv=*)
      # headline bench, default vs with an environment assignment (e.g. DCP_WGRAD_STREAM=1), twice
      c=${step#benchenv=}
      for r in 1 2; do
        timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/benchenv_default_$r.log 2>&1
        echo "default: $(grep -o '"value": [0-9.]*' $O/benchenv_default_$r.log)"
        env "$c" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/benchenv_set_$r.log 2>&1
        echo "$c: $(grep -o '"value": [0-9.]*' $O/benchenv_set_$r.log)"
      done ;;
    blas)
      timeout -k 10 300 python -u tools/blas_ref_bench.py --batch 1024 --iters 10 > $O/blas_ref_b1024.txt 2>&1
      tail -2 $O/blas_ref_b1024.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu_round $T done"
