#!/bin/bash
# round-2 probes: library GEMM ceiling, counter list, kernel stats of the graph-mode step
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 40 "gpurun_out/$name.log"; [ "$rc" -lt 124 ] || exit "$rc"; }
for s in "$@"; do
  case "$s" in
    blas) step blas 300 python tools/blas_ref.py ;;
    gemmt) step gemmt 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -m gpu -k "gemm" ;;
    blasdbg) step blasdbg 400 python tools/blas_ref.py --dbg 0,1,9 --variants p3,p3+16,p4 --nobias --only "qkv fwd,ffn1 fwd,ffn2 fwd,out fwd,ffn2 dgrad,ffn1 dgrad" ;;
    pmcg) for f in 0 9; do step pmcg$f 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmcg$f -o run --output-format csv -- python3 tools/blas_ref.py --dbg $f --only "ffn1 fwd" --variants p4 --nobias --nogrouped --noblas --reps 5 --rounds 2; done ;;
    gemmt16) ASRX_GEMM_DBG=16 step gemmt16 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -m gpu -k "gemm" ;;
    parity) step parity 600 python -u -m pytest tests/test_gpu_train_parity.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread -m gpu ;;
    benchab) for k in p3 p4 p3 p4; do ASRX_WGRAD_KIND=$k step bench_$k 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$k.log; done ;;
    other) step other 400 python -c "import bench, json; print(json.dumps(bench.other_configs()))" ;;
    attnt) step attnt 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -m gpu -k "attention" ;;
    blasepi) step blasepi 300 python tools/blas_ref.py --dbg 0,1 --variants p3,p4 --nobias --nogrouped --only "ffn1 fwd epi,ffn2 dgrad gated,ffn1 fwd,qkv fwd" ;;
    decode) step decode 600 python -u -m pytest tests/test_gpu_model.py -x -v --timeout 300 --timeout-method thread -m gpu -k "greedy" ;;
    feat) step feat 300 python -u -m pytest tests/test_features.py -x -v --timeout 120 --timeout-method thread -m gpu ;;
    pmcs) step pmcs 300 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d gpurun_out/pmcs -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-probe --no-sub --no-other ;;
    wg) step wg 400 python tools/blas_ref.py --dbg 0,9 --only none --wgrad p4,p5 ;;
    benchw) for k in p4 p5 p4 p5; do ASRX_WGRAD_KIND=$k step bench_$k 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$k.log; grep -o '"avg_launch_us": [0-9.]*' gpurun_out/bench_$k.log; done ;;
    pmcft) step pmcf 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-probe --no-sub --no-other && step pmcw 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-probe --no-sub --no-other && python3 tools/pmc_traffic.py gpurun_out/pmcf/run_counter_collection.csv gpurun_out/pmcw/run_counter_collection.csv c3 gpurun_out/c3_pmc_traffic.json ;;
    gtest) step gtest 400 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -m gpu -k "graphed" ;;
    attnb) step attnb 300 python tools/attn_bench.py ;;
    attndbg) step attndbg 300 python tools/attn_bench.py --dbg --only enc,cross ;;
    smx) step smx 300 python tools/softmax_probe.py ;;
    ln) step ln 300 python tools/ln_bench.py --blocks 256,512,1024,2048 ;;
    counters) step counters 120 rocprofv3 -L ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-probe --no-sub --no-other ;;
    pmcm) step pmcm 300 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmcm -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-probe --no-sub --no-other && python3 tools/pmc_mfma.py gpurun_out/pmcm/run_counter_collection.csv --out gpurun_out/c3_pmc_mfma.json ;;
    newt) step newt 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu -k "hipblaslt or adam" ;;
    blasres) step blasres 300 python tools/blas_ref.py --variants p3 --nogrouped --only "ffn2 fwd res,dec ffn2 fwd res,out fwd res,dec ffn1 dg512,dec qkv dg512,enc qkv dg512,dec out dg512" ;;
    abm) bash tools/ab_env.sh 2 ASRX_GEMM_BLASLT_M=8192 ASRX_GEMM_BLASLT_M=4096 || exit $? ;;
    abp4) bash tools/ab_env.sh 2 ASRX_P4_MIN_TILES=320 ASRX_P4_MIN_TILES=400 || exit $? ;;
    blasqkv) ASRX_P4_MIN_TILES=400 step blasqkv 300 python tools/blas_ref.py --variants p3,p4,auto --nogrouped --noblas --only "qkv fwd" ;;
    abpack) bash tools/ab_env.sh 2 ASRX_WGRAD_PACK=0 ASRX_WGRAD_PACK=1 || exit $? ;;
    steptab) python3 tools/step_table.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/step_table.txt && head -45 gpurun_out/step_table.txt ;;
    distt) step distt 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 500 --timeout-method thread -m gpu ;;
    rehearse) ASRX_DP_REHEARSE=1 step rehearse 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other && ASRX_DP_REHEARSE=1 ASRX_DP_WIRE=bf16 step rehearse_bf16 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other ;;
    abrel) for v in 6 0 6 0; do ASRX_DP_REHEARSE=1 ASRX_DP_RELEASE_LAYERS=$v step rel$v 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other; grep -o '"ms_per_step": [0-9.]*\|"launches_per_step": [0-9]*\|"avg_launch_us": [0-9.]*\|"allreduce_exposed_ms_per_rank": [^]]*' gpurun_out/rel$v.log | tr '\n' ' '; echo; done ;;
    abpackdp) for v in 0 1; do ASRX_DP_REHEARSE=1 ASRX_WGRAD_PACK=$v step packdp$v 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other; grep -o '"ms_per_step": [0-9.]*\|"launches_per_step": [0-9]*\|"avg_launch_us": [0-9.]*\|"host_enqueue_ms_per_step": [0-9.]*' gpurun_out/packdp$v.log | tr '\n' ' '; echo; done ;;
    profdp) ASRX_DP_REHEARSE=1 step profdp 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profdp -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-probe --no-sub --no-other && python3 tools/step_table.py gpurun_out/profdp/run_kernel_trace.csv > gpurun_out/steptab_dp.txt && head -30 gpurun_out/steptab_dp.txt ;;
    pmcsub) step pmcsf 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcsf -o run --output-format csv -- python3 tools/sub_pmc.py && step pmcsw 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcsw -o run --output-format csv -- python3 tools/sub_pmc.py && step pmcsj 120 python3 tools/pmc_traffic.py gpurun_out/pmcsf/run_counter_collection.csv gpurun_out/pmcsw/run_counter_collection.csv sub gpurun_out/sub_pmc_traffic.json && cat gpurun_out/sub_pmc_traffic.json | head -60 ;;
    m4096) for kv in "ASRX_GEMM_BLASLT_M=4096 ASRX_GEMM_BLASLT_RESID=0" "ASRX_GEMM_BLASLT_M=4096" "ASRX_GEMM_BLASLT_M=8192"; do env $kv timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other > gpurun_out/m4096.log 2>&1 || exit $?; echo "$kv $(grep -o '"ms_per_step": [0-9.]*\|"host_enqueue_ms_per_step": [0-9.]*' gpurun_out/m4096.log | tr '\n' ' ')"; done; ASRX_GEMM_BLASLT_M=4096 step profm 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profm -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-probe --no-sub --no-other && python3 tools/step_table.py gpurun_out/profm/run_kernel_trace.csv > gpurun_out/steptab_m.txt && head -12 gpurun_out/steptab_m.txt ;;
    abearly) for v in 0 1 0 1; do ASRX_DP_REHEARSE=1 ASRX_DP_EARLY_ADAM=$v step early$v 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-sub --no-other; echo "early=$v $(grep -o '"ms_per_step": [0-9.]*\|"allreduce_exposed_ms_per_rank": [^]]*' gpurun_out/early$v.log | tr '\n' ' ')"; done ;;
    smt) step smt 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu -k "softmax" ;;
    abres) bash tools/ab_env.sh 2 ASRX_GEMM_BLASLT_RESID=0 ASRX_GEMM_BLASLT_RESID=1 || exit $? ;;
    gpu) step gputests 1000 python -u -m pytest tests -x -q --timeout 400 --timeout-method thread -m gpu ;;
    *) echo "unknown $s"; exit 2 ;;
  esac
done

