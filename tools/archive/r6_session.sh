#!/bin/bash
# round-6 GPU session: STEPS (default "tests bench prof") with per-step time limits; stops at the first failure
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${SESSION:-r6}; mkdir -p $O
# a failing step ends the session, except pytest's "some tests failed" (exit 1): assertion failures are no GPU
# fault, so the benches after it still run; timeouts, aborts and crashes (124, 137, 134, 139, ...) end it
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  if [ $rc -eq 1 ] && [ "${name#t}" != "$name" ]; then return 0; fi
  [ $rc -ne 0 ] && exit $rc; return 0; }
export TMPDIR=/tmp
for s in ${STEPS:-tests bench prof}; do
  case $s in
    tests) run tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TESTSEL:+-k "$TESTSEL"} ;;
    tfile) run tfile 600 python -u -m pytest ${TFILES} -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    bench) run bench 300 python bench.py --steps ${BSTEPS:-20} --warmup 3 --no-cpu-baseline ;;
    abfrozen) for r in 1 2; do
             run fa_on_$r 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --plain-line off --frozen-ahead
             run fa_off_$r 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --plain-line off
             run fa_str_$r 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --plain-line off --frozen-ahead --frozen-stream
             run fa_pipe_$r 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --plain-line off --frozen-pipe
             run fs_on_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --dp-path --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --frozen-ahead
             run fs_off_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --dp-path --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run fs_str_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --dp-path --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --frozen-ahead --frozen-stream
             run fs_pipe_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --dp-path --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --frozen-pipe
           done ;;
    benchcpu) run benchcpu 400 python bench.py --steps ${BSTEPS:-20} --warmup 3 ;;
    plain) run plain 300 python bench.py --api plain --steps 20 --warmup 3 --no-cpu-baseline --no-roofline ;;
    plainall) run plain 300 python bench.py --api plain --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
              run plain_nodefer 300 python bench.py --api plain --no-defer-jets --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
              run plain_M 300 python bench.py --api plain --config fluid2DtlgnM --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
              run plain_adv 300 python bench.py --api plain --config advect1D --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
              run fused_adv 300 python bench.py --config advect1D --steps 20 --warmup 3 --no-cpu-baseline --no-roofline ;;
    configs) for c in ${CONFIGS:-advect1D elasticity2Dstretch elasticity3Dbunny fluid2DtlgnM}; do
               run bench_$c 400 python bench.py --config $c --steps ${CSTEPS:-10} --warmup 3 --no-cpu-baseline; done ;;
    shards) run shard_M8 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
            run shard_el3d8 300 python bench.py --config elasticity3Dbunny --shard-of 8 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline ;;
    dpshard) run dpshard_M8 300 python bench.py --config fluid2DtlgnM --shard-of 8 --dp-path --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
             run dpshard_el3d8 300 python bench.py --config elasticity3Dbunny --shard-of 8 --dp-path --steps 10 --warmup 3 --no-cpu-baseline --no-roofline ;;
    pol4) run pol4_shard 300 python bench.py --config fluid2DtlgnM --shard-of 8 --bwd-policy 4 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
          run pol4_head 300 python bench.py --bwd-policy 4 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline ;;
    abseeddp) for r in 1 2; do
             run sdp_A_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --dp-path --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run sdp_B_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --dp-path --no-seed-in-bwd --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
           done ;;
    profdp) run profdp 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profdp" -o run --output-format csv -- python bench.py --config fluid2DtlgnM --shard-of 8 --dp-path --steps 10 --warmup 3 --no-cpu-baseline --no-roofline ;;
    ablib) for r in 1 2; do
             run ab_A_$r 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run ab_B_$r 300 python bench.py --lib insr-pde_amd/lib_exp/libinsr_hip.so --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run ab_As_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run ab_Bs_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --lib insr-pde_amd/lib_exp/libinsr_hip.so --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
           done ;;
    abseed) for r in 1 2; do
             run sd_A_$r 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run sd_B_$r 300 python bench.py --no-seed-in-bwd --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run sd_As_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run sd_Bs_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --no-seed-in-bwd --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
           done ;;
    prof) run prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof" -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
    profB) run profB 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profB" -o run --output-format csv -- python bench.py --no-seed-in-bwd --steps 20 --warmup 3 --no-cpu-baseline ;;
    profshardB) run profshardB 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profshardB" -o run --output-format csv -- python bench.py --config fluid2DtlgnM --shard-of 8 --no-seed-in-bwd --steps 10 --warmup 3 --no-cpu-baseline --no-roofline ;;
    profadvplain) run profadvplain 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profadvplain" -o run --output-format csv -- python bench.py --api plain --config advect1D --steps 20 --warmup 3 --no-cpu-baseline --no-roofline ;;
    pmc) PRX='jet_|dw_x6|reduce_'  # HBM bytes per dispatch (eager run): FETCH_SIZE, WRITE_SIZE and SQ in passes of their own
         run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$PRX" -d "$PWD/$O/pmc_fetch" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-roofline
         run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$PRX" -d "$PWD/$O/pmc_write" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-roofline
         run pmc_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "$PRX" -d "$PWD/$O/pmc_sq" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-roofline ;;
    profplain) run profplain 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profplain" -o run --output-format csv -- python bench.py --api plain --steps 10 --warmup 3 --no-cpu-baseline --no-roofline ;;
    profshard) run profshard 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profshard" -o run --output-format csv -- python bench.py --config fluid2DtlgnM --shard-of 8 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline ;;
    kbench) run kbench 400 python tools/kbench.py ${KARGS:---sizes 8192,16708,66844 --nets fluid_pres --modes lap --variants h3 --policies 0,2} ;;
    profel) run profel_plain 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profel_plain" -o run --output-format csv -- python bench.py --api plain --config elasticity2Dstretch --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
            run profel_fused 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profel_fused" -o run --output-format csv -- python bench.py --config elasticity2Dstretch --steps 10 --warmup 3 --no-cpu-baseline --no-roofline ;;
    cpustudy) run cpustudy 400 python -u tools/cpu_leg_study.py ${CPUSEC:-8} ;;
    plainel) run plain_el2d 300 python bench.py --api plain --config elasticity2Dstretch --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
             run fused_el2d 300 python bench.py --config elasticity2Dstretch --steps 10 --warmup 3 --no-cpu-baseline --no-roofline ;;
    pmcel3d) PRX='jet_|dw_x6|reduce_'
         run pmcel_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$PRX" -d "$PWD/$O/pmcel_fetch" -o run --output-format csv -- python bench.py --config elasticity3Dbunny --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-roofline
         run pmcel_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$PRX" -d "$PWD/$O/pmcel_write" -o run --output-format csv -- python bench.py --config elasticity3Dbunny --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-roofline
         run pmcel_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "$PRX" -d "$PWD/$O/pmcel_sq" -o run --output-format csv -- python bench.py --config elasticity3Dbunny --steps 1 --warmup 1 --no-graph --no-cpu-baseline --no-roofline ;;
    advab) for r in 1 2; do
             run adv_fused_$r 300 python bench.py --config advect1D --steps 40 --warmup 3 --no-cpu-baseline
             run adv_generic_$r 300 python bench.py --config advect1D --steps 40 --warmup 3 --no-cpu-baseline --no-advect-fused
           done
           run adv_plain 300 python bench.py --api plain --config advect1D --steps 40 --warmup 3 --no-cpu-baseline --no-roofline ;;
    profadv) run profadv 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profadv" -o run --output-format csv -- python bench.py --config advect1D --steps 20 --warmup 3 --no-cpu-baseline ;;
    pmcall) PRX='jet_|dw_x6|reduce_|advect1d'  # per config: FETCH_SIZE, WRITE_SIZE, SQ in passes of their own
         for spec in "head:" "adv:--config advect1D" "shard:--config fluid2DtlgnM --shard-of 8" "el2d:--config elasticity2Dstretch"; do
           nm=${spec%%:*}; ca=${spec#*:}
           for pass in fetch write sq; do
             case $pass in fetch) cnt="FETCH_SIZE";; write) cnt="WRITE_SIZE";;
               sq) cnt="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT";; esac
             run pmc_${nm}_$pass 300 rocprofv3 --pmc $cnt --kernel-include-regex "$PRX" -d "$PWD/$O/$nm/pmc_$pass" -o run --output-format csv -- python bench.py $ca --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-roofline
           done
         done ;;
    abel) for r in 1 2; do
             run el_res_$r 300 python bench.py --config elasticity2Dstretch --steps 20 --warmup 3 --no-cpu-baseline
             run el_2k_$r 300 python bench.py --config elasticity2Dstretch --steps 20 --warmup 3 --no-cpu-baseline --bwd-policy 2
           done
           run el_plain 300 python bench.py --api plain --config elasticity2Dstretch --steps 20 --warmup 3 --no-cpu-baseline --no-roofline ;;
    abpol5) for r in 1 2; do
             run p0_head_$r 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --plain-line off
             run p5_head_$r 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --plain-line off --bwd-policy 5
             run p0_shard_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run p5_shard_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --bwd-policy 5
           done
           run p0_M 300 python bench.py --config fluid2DtlgnM --steps 20 --warmup 3 --no-cpu-baseline
           run p5_M 300 python bench.py --config fluid2DtlgnM --steps 20 --warmup 3 --no-cpu-baseline --bwd-policy 5 ;;
    default) run default 600 python bench.py ;;
    tfb) run tfb 900 python -u -m pytest tests/test_gpu_resident_f16.py tests/test_gpu_multi_bwd.py tests/test_gpu_recompute.py tests/test_gpu_seeds.py tests/test_gpu_phases.py tests/test_gpu_fullsize_phases.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
    abpol4) for r in 1 2; do
              run p0h_$r 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --plain-line off
              run p4h_$r 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --plain-line off --bwd-policy 4
              run p0s_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
              run p4s_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --bwd-policy 4
            done
            run p4prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/p4prof" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --plain-line off --bwd-policy 4 ;;
    topt) run topt 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_phases.py tests/test_gpu_fullsize_phases.py tests/test_gpu_dp_capture.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
    adamcost) run adamcost 300 python tools/study/adam_sums_cost.py ;;
    profshard) run profshard 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profshard" -o run --output-format csv -- python bench.py --config fluid2DtlgnM --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
               run profshardB 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profshardB" -o run --output-format csv -- python bench.py --config fluid2DtlgnM --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --lib insr-pde_amd/lib_exp/libinsr_hip.so ;;
    t3) run tt3 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_multi_bwd.py tests/test_gpu_fullsize_phases.py tests/test_gpu_phases.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
    advf16) run tadv 600 python -u -m pytest tests/test_gpu_advect_iter.py tests/test_gpu_fullsize_phases.py -m gpu -x -v --timeout 120 --timeout-method thread -k "advect"
            for r in 1 2; do
              run adv16_$r 300 python bench.py --config advect1D --steps 40 --warmup 3 --no-cpu-baseline
              run adv32_$r 300 python bench.py --config advect1D --steps 40 --warmup 3 --no-cpu-baseline --advect-fp32
            done
            run advprof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/advprof" -o run --output-format csv -- python bench.py --config advect1D --steps 20 --warmup 3 --no-cpu-baseline --no-roofline ;;
    abx) for r in 1 2; do  # this tree's library (A) vs insr-pde_amd/lib_exp (B: the previous build)
           run x_A_$r 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --plain-line off
           run x_B_$r 300 python bench.py --lib insr-pde_amd/lib_exp/libinsr_hip.so --steps 40 --warmup 3 --no-cpu-baseline --plain-line off
           run x_As_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
           run x_Bs_$r 300 python bench.py --config fluid2DtlgnM --shard-of 8 --lib insr-pde_amd/lib_exp/libinsr_hip.so --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
         done
         run x_prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/xprof" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --plain-line off ;;
    closing) run bench_advect1D 300 python bench.py --config advect1D --steps 40 --warmup 3 --no-cpu-baseline
             for c in elasticity2Dstretch elasticity3Dbunny fluid2DtlgnM; do
               run bench_$c 400 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline; done
             run shard_M8 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run dpshard_M8 300 python bench.py --config fluid2DtlgnM --shard-of 8 --dp-path --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run shard_el3d8 300 python bench.py --config elasticity3Dbunny --shard-of 8 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
             run dpshard_el3d8 300 python bench.py --config elasticity3Dbunny --shard-of 8 --dp-path --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
             run plain_el2d 300 python bench.py --api plain --config elasticity2Dstretch --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
             run plain_adv 300 python bench.py --api plain --config advect1D --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
             run plain_M 300 python bench.py --api plain --config fluid2DtlgnM --steps 20 --warmup 3 --no-cpu-baseline --no-roofline ;;
    prec) run prec 400 python tools/prec_errors.py ${PARGS:-} ;;
    precd) run precd 900 python -u tools/prec_defaults.py ${PDARGS:-} ;;
  esac
done
echo done >> $O/status.log
