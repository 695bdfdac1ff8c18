#!/bin/bash
# Named GPU steps for one gpurun call (round 3 on), e.g.
#   gpurun --timeout 900 -- bash scripts/gpu_steps.sh OUT=gpurun_out/r3a tests smoke bench20
# Every step runs under its own time limit, logs to $OUT/<step>.log, and the
# chain stops at the first failure, fault or timeout (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=gpurun_out/steps
for a in "$@"; do case $a in OUT=*) OUT=${a#OUT=} ;; esac; done
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name start $(date +%T)"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"; tail -3 "$OUT/$name.log" | cut -c1-300
  return $rc
}
prof() {  # name timeout rocprofv3-args... -- cmd...
  local name=$1 t=$2; shift 2
  echo "== $name start $(date +%T)"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 "$t" rocprofv3 "$@" > "$R/$OUT/$name.log" 2>&1)
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"; tail -3 "$OUT/$name.log" | cut -c1-300
  return $rc
}
for s in "$@"; do
  case $s in
    OUT=*) ;;
    # the driver's exact GPU-suite command (pytest.ini: timeout 900, signal method)
    tests) step tests 1000 python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider || exit 1 ;;
    tests_new) step tests_new 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
             tests/test_bench_gpu.py tests/test_drift_gpu.py \
             "tests/test_multirank_gpu.py::test_aligned_frames_on_partial_sides_bitwise" \
             "tests/test_multirank_gpu.py::test_aligned_frames_with_ol_bands_bitwise" || exit 1 ;;
    tests_capi) step tests_capi 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
             tests/test_capi_gpu.py || exit 1 ;;
    tests_pipe) step tests_pipe 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
             tests/test_pipe_gpu.py -p no:cacheprovider || exit 1 ;;
    sweep5) step sweep5 600 python bench/pass_sweep.py --n 101120 --rounds 5 --pipe 16,20,24 \
             --pipe5 16-20 --pipec "" --ldsdpp "" --old "" --alt "" --out "$OUT/sweep5.json" || exit 1 ;;
    sweep5b) step sweep5b 600 python bench/pass_sweep.py --n 101120 --rounds 5 --pipe 20,24 \
             --pipe5 20 --chunks5 20:1536/2048/4096 --kinds piper:20,piper:24,pipe_diag1:20,pipe_diag1:24 \
             --pipec "" --ldsdpp "" --old "" --alt "" --out "$OUT/sweep5b.json" || exit 1 ;;
    pmc5a) prof pmc5a 300 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
             SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
             --output-format csv -d "$R/$OUT/pmc5a" -o run -- python3 "$R/bench/pass_sweep.py" \
             --n 101120 --rounds 2 --pipe 20,24 --pipe5 20 --kinds pipe_diag1:24 --pipec "" \
             --ldsdpp "" --old "" --alt "" || exit 1 ;;
    sweepr) step sweepr 600 python bench/pass_sweep.py --n 101120 --rounds 5 --pipe 12,16,20,24 \
             --pipe5 20 --kinds piper:12,piper:16,piper:20,piper:24,pipe_diag1:24 \
             --pipec "" --ldsdpp "" --old "" --alt "" --out "$OUT/sweepr.json" || exit 1 ;;
    sweepr2) step sweepr2 600 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe 16,20,24 \
             --pipe5 20 --kinds piper:20,piper:24 \
             --pipec "" --ldsdpp "" --old "" --alt "" --out "$OUT/sweepr2.json" || exit 1 ;;
    bench20_pipe|bench20_piper|bench20_pipe5) v=${s#bench20_}
             RMA_PIPE_FAST=$v step "$s" 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
             --json-out "$OUT/$s.json" || exit 1 ;;
    bench1000_pipe|bench1000_piper) v=${s#bench1000_}
             RMA_PIPE_FAST=$v step "$s" 300 python bench.py --json-out "$OUT/$s.json" || exit 1 ;;
    sweepr3) step sweepr3 600 python bench/pass_sweep.py --n 101120 --rounds 5 --pipe 17,18,19,20,24 \
             --kinds piper:17,piper:18,piper:19,piper:20 \
             --pipec "" --ldsdpp "" --old "" --alt "" --out "$OUT/sweepr3.json" || exit 1 ;;
    sweepg) step sweepg 600 python bench/pass_sweep.py --n 101120 --rounds 5 --pipe 20,21,22,23,24 \
             --kinds piper:20,piper:21,piper:22,piper:23,piper:24,pipe_diag1:24 \
             --pipec "" --ldsdpp "" --old "" --alt "" --out "$OUT/sweepg.json" || exit 1 ;;
    pmcg) prof pmcg 300 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
             SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
             --output-format csv -d "$R/$OUT/pmcg" -o run -- python3 "$R/bench/pass_sweep.py" \
             --n 101120 --rounds 1 --pipe 20,24 --kinds piper:20,piper:24,pipe_diag1:24 --pipec "" \
             --ldsdpp "" --old "" --alt "" || exit 1 ;;
    sweepg_small) step sweepg_small 600 python bench/pass_sweep.py --n 16384 --rounds 7 \
             --pipe 17,20,24 --kinds piper:17,piper:20,piper:24 --pipec "" --ldsdpp "" --old "" \
             --alt "" --out "$OUT/sweepg_16384.json" && \
             step sweepg_4096 600 python bench/pass_sweep.py --n 4096 --rounds 9 \
             --pipe 17,20,24 --kinds piper:17,piper:20,piper:24 --pipec "" --ldsdpp "" --old "" \
             --alt "" --out "$OUT/sweepg_4096.json" || exit 1 ;;
    sweepc) step sweepc 600 python bench/pass_sweep.py --n 101120 --rounds 5 --pipe 20,24 \
             --kinds piper:20,piper:20:2048,piper:20:4096,piper:20:6144,piper:24,piper:24:2048,piper:24:4096,piper:24:6144 \
             --pipec "" --ldsdpp "" --old "" --alt "" --out "$OUT/sweepc.json" || exit 1 ;;
    prof20) prof prof20 300 --kernel-trace --stats -d "$R/$OUT/prof20" -o run -- python3 \
             "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --json-out "$R/$OUT/prof20.json" || exit 1 ;;
    sweeplo) step sweeplo 600 python bench/pass_sweep.py --n 101120 --rounds 5 --pipe 10,12,14,16,17,18 \
             --kinds piper:10,piper:12,piper:14,piper:16,piper:17,piper:18 \
             --pipec "" --ldsdpp "" --old "" --alt "" --out "$OUT/sweeplo.json" && \
             step sweeplo16k 600 python bench/pass_sweep.py --n 16384 --rounds 7 --pipe 10,12,14,16 \
             --kinds piper:10,piper:12,piper:14,piper:16 \
             --pipec "" --ldsdpp "" --old "" --alt "" --out "$OUT/sweeplo16k.json" || exit 1 ;;
    prof_host4096) prof prof_host4096 300 --kernel-trace --output-format csv -d "$R/$OUT/prof_host4096" \
             -o run -- python3 "$R/bench/rccl_self_overhead.py" --n 4096 --K 1 --variants perf_hide \
             --steps 200 --pattern op --out "$R/$OUT/prof_host4096.json" || exit 1 ;;
    host4096_nocross) RMA_HALO_CROSS=0 step host4096_nocross 300 python bench/rccl_self_overhead.py \
             --n 4096 --K 1 --variants perf_hide --steps 400 --pattern opop \
             --out "$OUT/host4096_nocross.json" || exit 1 ;;
    host4096_ch4|host4096_ch8|host4096_ch16) c=${s#host4096_ch}
             NCCL_MIN_P2P_NCHANNELS=$c NCCL_MAX_P2P_NCHANNELS=$c step "$s" 300 python \
             bench/rccl_self_overhead.py --n 4096 --K 1 --variants perf_hide --steps 400 --pattern opop \
             --out "$OUT/$s.json" || exit 1 ;;
    bench6000) step bench6000 400 python bench.py --steps 6000 --warmup 24 \
             --json-out "$OUT/bench6000.json" || exit 1 ;;
    pmc_bytes) prof pmc_fetch 300 --pmc FETCH_SIZE SQ_WAVES GRBM_GUI_ACTIVE \
             --output-format csv -d "$R/$OUT/pmc_fetch" -o run -- python3 "$R/bench/pass_sweep.py" \
             --n 101120 --rounds 1 --pipe 24 --kinds piper:24 --pipec "" \
             --ldsdpp "" --old "" --alt "" && \
             prof pmc_write 300 --pmc WRITE_SIZE SQ_WAVES GRBM_GUI_ACTIVE \
             --output-format csv -d "$R/$OUT/pmc_write" -o run -- python3 "$R/bench/pass_sweep.py" \
             --n 101120 --rounds 1 --pipe 24 --kinds piper:24 --pipec "" \
             --ldsdpp "" --old "" --alt "" || exit 1 ;;
    sweepc2) step sweepc2 600 python bench/pass_sweep.py --n 101120 --rounds 5 --pipe "" \
             --kinds piper:20:2560,piper:20:2816,piper:20,piper:20:3328,piper:20:3584,piper:24:2816,piper:24,piper:24:3328 \
             --pipec "" --ldsdpp "" --old "" --alt "" --out "$OUT/sweepc2.json" || exit 1 ;;
    coef_ab) step coef_ab 400 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" --coef-dims 4,2 --coef-alt 1,1 \
             --kinds piper:20,piper:24,piper6:20,piper6:24,piper7:20,piper7:24 \
             --out "$OUT/coef_ab.json" || exit 1 ;;
    u6_ab) step u6_ab 400 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" \
             --kinds piper:17,piper:18,piper:19,piper:20,piper_u3:17,piper_u3:18,piper_u3:19,piper_u3:20 \
             --out "$OUT/u6_ab.json" || exit 1 ;;
    iso_ab) step iso_ab 400 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" --coef-dims 1,1 \
             --kinds piper:20,piper:24,piper_iso:20,piper_iso:24,piper_u3:20 \
             --out "$OUT/iso_ab.json" || exit 1 ;;
    eqsmall) for t in eqn4096_x eqn4096_x_cd2 eqn4096_xy eqn4096_xy_cd2 eqn4096_xy_strips \
                      eqn8192_xy eqn8192_xy_cd2; do bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    eqsmall2) for t in eqn4096_xy_cd2_bol eqn4096_xy_bol eqn4096_xy_cd4_bol eqn4096_x_cd4 \
                      eqn4096_y eqn4096_y_cd2 eqn4096_y_bol eqn8192_xy_cd4 eqn8192_xy_cd2_bol \
                      eqn8192_x eqn8192_x_cd2 eqn8192_y eqn8192_y_cd2 eqn16384_xy eqn16384_xy_cd2 \
                      eqn2048_xy eqn2048_xy_cd2 eqn2048_xy_strips; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    eqdefault) for t in eqn4096_x eqn4096_y eqn4096_xy eqn8192_x eqn8192_y eqn8192_xy eqn16384_xy; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    tests_frames) step tests_frames 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
             "tests/test_multirank_gpu.py" -p no:cacheprovider || exit 1 ;;
    chunk20) step chunk20 600 python bench/pass_sweep.py --n 101120 --rounds 5 --pipe "" \
             --kinds piper:20:2560,piper:20:2816,piper:20:2890,piper:20:2976,piper:20,piper:20:3160,piper:20:3328 \
             --pipec "" --ldsdpp "" --old "" --alt "" --out "$OUT/chunk20.json" || exit 1 ;;
    u6_small) for n in 16384 8192 4096; do
               step u6_$n 600 python bench/pass_sweep.py --n $n --rounds 9 --pipe "" --pipec "" \
               --ldsdpp "" --old "" --alt "" \
               --kinds piper:17,piper:18,piper:19,piper:20,piper_u3:17,piper_u3:18,piper_u3:19,piper_u3:20 \
               --out "$OUT/u6_$n.json" || exit 1; done ;;
    exec_costs) for n in 101120 16384 8192 4096; do
               step exec_$n 600 python bench/pass_sweep.py --n $n --rounds 7 --pipe "" --pipec "" \
               --ldsdpp "" --old "" --alt "" --exec 1-24 --out "$OUT/exec_$n.json" || exit 1; done ;;
    diag_s0) step diag_s0 400 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" --kinds piper:20,piper_diag_s0:20 \
             --out "$OUT/diag_s0.json" || exit 1 ;;
    trace8192y) prof trace8192y 300 --kernel-trace --output-format csv -d "$R/$OUT/trace8192y" \
             -o run -- python3 "$R/bench/rccl_self_overhead.py" --n 8192 --K 24 --variants perf_hide \
             --periodic y --steps 480 --pattern op --spacing equal --out "$R/$OUT/trace8192y.json" || exit 1 ;;
    eqsmall3) for t in eqn8192_y_bol eqn8192_y_cd2_bol eqn8192_y_cd3 eqn8192_y_cd4_bol eqn8192_xy_bol \
                      eqn8192_xy_cd3 eqn8192_xy_cd4_bol eqn8192_y eqn8192_y_cd2 eqn16384_x eqn16384_y; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    eqmerge) for t in eqn2048_xy eqn2048_xy_nomerge eqn4096_xy eqn4096_xy_nomerge eqn8192_xy \
                      eqn8192_xy_nomerge eqn16384_xy eqn16384_xy_nomerge; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    eq_xy_nomerge) RMA_HALO_MERGED=0 step eq_xy_nomerge 400 python bench/rccl_self_overhead.py \
             --K 24 --periodic xy --steps 320 --pattern opop --spacing equal \
             --out "$OUT/eq_xy_nomerge.json" || exit 1 ;;
    tests_merge) step tests_merge 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
             tests/test_multirank_gpu.py tests/test_capi_gpu.py tests/test_bench_gpu.py \
             -p no:cacheprovider || exit 1 ;;
    eqchan) for t in eqn8192_xy eqn8192_xy_ch1 eqn8192_xy_ch2 eqn8192_xy_pp1 eqn4096_xy \
                     eqn4096_xy_ch1 eqn16384_xy eqn16384_xy_ch1; do
             bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    eqlag) for t in eqn2048_xy eqn2048_xy_nolag eqn4096_xy eqn4096_xy_nolag eqn4096_x eqn4096_x_nolag \
                    eqn8192_xy eqn8192_xy_nolag eqn16384_xy eqn16384_xy_nolag; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    w1_ab) step w1_ab 400 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" \
             --kinds piper:20,piper_w1:20,piper:24,piper_w1:24 --out "$OUT/w1_ab.json" || exit 1 ;;
    mask_ab) step mask_ab 400 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" \
             --kinds piper:20,piper_mask:20,piper_mask_ctl:20,piper:24,piper_mask:24,piper_mask_ctl:24 --out "$OUT/mask_ab.json" || exit 1 ;;
    nosb_ab) step nosb_ab 400 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" \
             --kinds piper:20,piper_nosb:20,piper:24,piper_nosb:24 --out "$OUT/nosb_ab.json" || exit 1 ;;
    tests_user) step tests_user 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
             "tests/test_multirank_gpu.py::test_user_example_gpu_equals_golden" -p no:cacheprovider && \
             step user_example 120 python examples/diffusion_2D_user.py --nx 8192 --ny 8192 --nt 200 && \
             step user_example_hide 120 python examples/diffusion_2D_user.py --nx 8192 --ny 8192 \
               --nt 200 --hide || exit 1 ;;
    pmc_u6) prof pmc_u6 240 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
             SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
             --output-format csv -d "$R/$OUT/pmc_u6" -o run -- python3 "$R/bench/pass_sweep.py" \
             --n 101120 --rounds 1 --pipe "" --pipec "" --ldsdpp "" --old "" --alt "" \
             --kinds piper:20,piper_u3:20,piper:24 || exit 1 ;;
    rot_ab) step rot_ab 400 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" \
             --kinds piper:20,piper_rot:20,piper:24,piper_rot:24 --out "$OUT/rot_ab.json" || exit 1 ;;
    prio_ab) step prio_ab 500 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" \
             --kinds piper:20,piper_rot:20,piper_prio:20,piper_prio_nr:20,piper:24,piper_prio:24 \
             --out "$OUT/prio_ab.json" || exit 1 ;;
    hb_ab) step hb_ab 400 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" \
             --kinds piper:20,piper_diag_hb:20 --out "$OUT/hb_ab.json" || exit 1 ;;
    u6s_ab) step u6s_ab 400 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" \
             --kinds piper:21,piper_u6s:21,piper:24,piper_u6s:24 --out "$OUT/u6s_ab.json" || exit 1 ;;
    sp_ab) step sp_ab 400 python bench/pass_sweep.py --n 101120 --rounds 7 --pipe "" \
             --pipec "" --ldsdpp "" --old "" --alt "" \
             --kinds piper:20,piper_sp:20,piper_sp2:20,piper:24,piper_sp:24,piper_sp2:24 \
             --out "$OUT/sp_ab.json" || exit 1 ;;
    tests_ipc) step tests_ipc 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
             "tests/test_multirank_gpu.py::test_ipc_transport_processes" \
             "tests/test_multirank_gpu.py::test_ipc_transport_temporal_tiles" \
             "tests/test_multirank_gpu.py::test_ipc_ring_smoke_test" \
             "tests/test_multirank_gpu.py::test_ipc_mailbox_overflow_fails_on_every_rank" \
             "tests/test_multirank_gpu.py::test_ipc_overflow_of_a_later_peer_keeps_the_transport_in_step" \
             "tests/test_multirank_gpu.py::test_ipc_update_halo_device_fields" \
             -p no:cacheprovider || exit 1 ;;
    ipc_modes) for mode in stream host; do
               for cfg in "258 1 2000" "1026 1 400" "2048 1 400" "4096 24 480"; do
                 set -- $cfg; tag="ipc_${mode}_$1_$2"
                 RMA_IPC_MODE=$mode step "$tag" 200 python -m rocm_mpi_amd.launch -n 4 -- \
                   bench/ipc_transport_probe.py --transport ipc --n $1 --K $2 --steps $3 || exit 1
               done
             done
             for cfg in "258 1 2000" "2048 1 400" "4096 24 480"; do
               set -- $cfg; tag="staged_$1_$2"
               step "$tag" 200 python -m rocm_mpi_amd.launch -n 4 -- \
                 bench/ipc_transport_probe.py --transport staged --n $1 --K $2 --steps $3 || exit 1
             done ;;
    ipc_graph) for cfg in "258 1 100" "2048 1 100" "4096 24 96"; do
               set -- $cfg
               for gr in "" "--graph"; do
                 tag="ipcg_$1_$2${gr:+_graph}"
                 RMA_IPC_MODE=stream step "$tag" 170 python -m rocm_mpi_amd.launch -n 4 -- \
                   bench/ipc_transport_probe.py --transport ipc --n $1 --K $2 --steps $3 --check $gr || exit 1
               done
             done ;;
    ipc_check24) for cfg in "ipc stream 1026 24 96" "ipc host 1026 24 96" "staged x 1026 24 96" \
                            "ipc stream 1026 8 96" "ipc stream 258 1 200"; do
               set -- $cfg; tag="chk_$1_$2_$3_$4"
               RMA_IPC_MODE=$2 step "$tag" 170 python -m rocm_mpi_amd.launch -n 4 -- \
                 bench/ipc_transport_probe.py --transport $1 --n $3 --K $4 --steps $5 --check; true
             done ;;
    ipc_cpwait) for cw in 1 0; do
               for cfg in "258 1 2000" "4096 24 480"; do
                 set -- $cfg; tag="ipc_stream_cpwait${cw}_$1_$2"
                 GPU_STREAMOPS_CP_WAIT=$cw RMA_IPC_MODE=stream step "$tag" 200 python -m rocm_mpi_amd.launch \
                   -n 4 -- bench/ipc_transport_probe.py --transport ipc --n $1 --K $2 --steps $3 --check || exit 1
               done
             done ;;
    fuzz_soak) step fuzz_soak 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
             tests/test_fuzz_gpu.py -p no:cacheprovider || exit 1 ;;
    tests_rccl_mp) step tests_rccl_mp 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
             "tests/test_multirank_gpu.py::test_rccl_ring_smoke_test_between_processes" \
             "tests/test_multirank_gpu.py::test_rccl_between_processes_sharing_the_gpu" \
             "tests/test_multirank_gpu.py::test_rccl_between_processes_temporal_tiles" \
             "tests/test_bench_gpu.py::test_bench_two_processes_sharing_the_gpu" \
             "tests/test_bench_gpu.py::test_bench_rehearsal_of_the_scaling_run_over_rccl" \
             -p no:cacheprovider || exit 1 ;;
    fuzz_procs) step fuzz_procs 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
             "tests/test_fuzz_gpu.py::test_random_decompositions_between_processes" \
             -p no:cacheprovider || exit 1 ;;
    presets_shared) step presets_shared 600 python bench/baseline_configs.py --shared-gpu --nt 120 \
             --out "$OUT/baseline_configs_shared.json" || exit 1 ;;
    rehearse) for n in 2 4 8; do
               step "rehearse$n" 400 python bench.py --gpus $n --shared-gpu-test --shared-gpu-transport rccl \
                 --nx 4096 --steps 96 --warmup 4 --json-out "$OUT/rehearse$n.json" || exit 1
             done ;;
    rehearse_fused) for n in 2 4 8; do
               step "rehearse_fused$n" 400 python bench.py --gpus $n --shared-gpu-test --shared-gpu-transport rccl \
                 --nx 8192 --steps 96 --warmup 4 --json-out "$OUT/rehearse_fused$n.json" || exit 1
             done ;;
    tests_ipc5) step tests_ipc5 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
             "tests/test_multirank_gpu.py::test_ipc_modes_2000_exchanged_steps_bitwise" \
             "tests/test_multirank_gpu.py::test_ipc_transport_processes" \
             "tests/test_multirank_gpu.py::test_ipc_transport_temporal_tiles" \
             "tests/test_multirank_gpu.py::test_ipc_ring_smoke_test" \
             "tests/test_multirank_gpu.py::test_ipc_mailbox_overflow_fails_on_every_rank" \
             "tests/test_multirank_gpu.py::test_ipc_overflow_of_a_later_peer_keeps_the_transport_in_step" \
             "tests/test_multirank_gpu.py::test_ipc_update_halo_device_fields" \
             -p no:cacheprovider || exit 1 ;;
    tests_ipc5g) step tests_ipc5g 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
             "tests/test_multirank_gpu.py::test_ipc_stream_mode_graph_replay_matches_golden" \
             -p no:cacheprovider || exit 1 ;;
    tests_ipc_ev) RMA_IPC_GPU_EVENTS=1 step tests_ipc_ev 400 python -u -m pytest -x -v --timeout 120 \
             --timeout-method thread "tests/test_multirank_gpu.py::test_ipc_transport_processes" \
             "tests/test_multirank_gpu.py::test_ipc_transport_temporal_tiles" -p no:cacheprovider || exit 1 ;;
    ipc_probe) for cfg in "ipc 258 1 2000 --check" "staged 258 1 2000 --check" "ipc 1026 1 400 --check" \
                          "ipc 2048 1 400" "staged 2048 1 400" "ipc 4096 24 480" "staged 4096 24 480"; do
               set -- $cfg; tag="ipc_probe_$1_$2_$3"
               step "$tag" 200 python -m rocm_mpi_amd.launch -n 4 -- bench/ipc_transport_probe.py \
                 --transport $1 --n $2 --K $3 --steps $4 $5 || exit 1
             done ;;
    tests_multirank) step tests_multirank 600 python -u -m pytest -x -q --timeout 120 \
             --timeout-method thread tests/test_multirank_gpu.py tests/test_executor_gpu.py \
             -p no:cacheprovider || exit 1 ;;
    tests_shared) step tests_shared 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
             "tests/test_bench_gpu.py::test_bench_two_processes_sharing_the_gpu" -p no:cacheprovider || exit 1 ;;
    chunk8192) for c in 128 192 256 384 512; do
               step "chunk8192_xy_$c" 300 python bench/rccl_self_overhead.py --n 8192 --K 24 \
                 --periodic xy --steps 2400 --pattern opop --spacing equal --chunk2 $c \
                 --out "$OUT/chunk8192_xy_$c.json" || exit 1
             done ;;
    apps_ipc) step ring_ipc 120 python -m rocm_mpi_amd.launch -n 4 -m \
               rocm_mpi_amd.apps.rocmaware_test_selectdevice -- --transport ipc && \
             step hide_ipc_2x2 300 python -m rocm_mpi_amd.launch -n 4 -m \
               rocm_mpi_amd.apps.diffusion_2D_perf_hide -- --transport ipc --nx 4096 --ny 4096 \
               --nt 1000 --dims 2,2 --device cuda:0 || exit 1 ;;
    ipc_trace) for t in ipc staged; do
               PYTHONPATH="$R" prof "ipc_trace_$t" 240 --memory-copy-trace --kernel-trace --stats --output-format csv \
                 -d "$R/$OUT/ipc_trace_$t" -o run -- python3 -m rocm_mpi_amd.launch -n 4 -- \
                 "$R/bench/ipc_transport_probe.py" --transport $t --n 258 --K 1 --steps 200 || exit 1
             done ;;
    tests_ipc_sf) RMA_IPC_STREAM_FLAGS=1 step tests_ipc_sf 400 python -u -m pytest -x -v --timeout 120 \
             --timeout-method thread "tests/test_multirank_gpu.py::test_ipc_transport_processes" \
             "tests/test_multirank_gpu.py::test_ipc_transport_temporal_tiles" \
             "tests/test_multirank_gpu.py::test_ipc_ring_smoke_test" -p no:cacheprovider || exit 1 ;;
    ipc_probe_sf) for cfg in "ipc 258 1 2000 --check" "ipc 2048 1 400" "ipc 4096 24 480"; do
               set -- $cfg; tag="ipc_probe_sf_$1_$2_$3"
               RMA_IPC_STREAM_FLAGS=1 step "$tag" 200 python -m rocm_mpi_amd.launch -n 4 -- \
                 bench/ipc_transport_probe.py --transport $1 --n $2 --K $3 --steps $4 $5 || exit 1
             done ;;
    bench_small) for n in 16384 8192 4096; do
               step "bench1000_$n" 300 python bench.py --nx $n --steps 1000 --json-out "$OUT/bench1000_$n.json" || exit 1
             done ;;
    tests_halo) step tests_halo 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
             tests/test_halo_gpu.py -p no:cacheprovider || exit 1 ;;
    tests_mask) step tests_mask 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
             "tests/test_pipe_gpu.py::test_piper_masked_cone_bitwise" \
             "tests/test_pipe_gpu.py::test_piper_schedule_variants_bitwise" \
             "tests/test_pipe_gpu.py::test_piper_u6_spilling_bitwise" -p no:cacheprovider || exit 1 ;;
    tests_w1) step tests_w1 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
             "tests/test_pipe_gpu.py::test_piper_one_wave_per_simd_bitwise" -p no:cacheprovider || exit 1 ;;
    apps_r4) step app_hide16k 300 python -m rocm_mpi_amd.apps.diffusion_2D_perf_hide --nx 16384 \
               --ny 16384 --nt 1000 --json && \
             step app_perf12k 300 python -m rocm_mpi_amd.apps.diffusion_2D_perf --nt 1000 --json && \
             step app_perf12k_canonical 300 python -m rocm_mpi_amd.apps.diffusion_2D_perf --nt 1000 \
               --canonical --json && \
             step app_perf12k_k1 300 python -m rocm_mpi_amd.apps.diffusion_2D_perf --nt 1000 \
               --temporal 1 --json && \
             step baseline_presets 600 python bench/baseline_configs.py --max-gpus 1 \
               --out "$OUT/baseline_configs.json" || exit 1 ;;
    tests_r4) step tests_r4 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
             tests/test_capi_gpu.py tests/test_bench_gpu.py "tests/test_pipe_gpu.py::test_piper_split_form_bitwise" \
             "tests/test_pipe_gpu.py::test_piper_unroll6_equals_unroll3" \
             "tests/test_pipe_gpu.py::test_piper_iso_bitwise_and_refused_when_anisotropic" \
             "tests/test_pipe_gpu.py::test_piper_register_factors_bitwise" \
             "tests/test_temporal_gpu.py::test_headline_kernels_beyond_2e31_cells" \
             -p no:cacheprovider || exit 1 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench20) step bench20 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
             --json-out "$OUT/bench20.json" || exit 1 ;;
    bench1000) step bench1000 300 python bench.py --json-out "$OUT/bench1000.json" || exit 1 ;;
    nbr_x|nbr_y|nbr_xy) d=${s#nbr_}
             step "$s" 400 python bench/rccl_self_overhead.py --K 24 --periodic "$d" --steps 320 \
             --pattern opop --out "$OUT/$s.json" || exit 1 ;;
    nbr_x_strips|nbr_y_strips|nbr_xy_strips) d=${s#nbr_}; d=${d%_strips}
             RMA_FRAME_ALIGNED=0 step "$s" 400 python bench/rccl_self_overhead.py --K 24 \
             --periodic "$d" --steps 320 --pattern opop --out "$OUT/$s.json" || exit 1 ;;
    eq_x|eq_y|eq_xy) d=${s#eq_}
             step "$s" 400 python bench/rccl_self_overhead.py --K 24 --periodic "$d" --steps 320 \
             --pattern opop --spacing equal --out "$OUT/$s.json" || exit 1 ;;
    eq_x_strips|eq_y_strips|eq_xy_strips) d=${s#eq_}; d=${d%_strips}
             RMA_FRAME_ALIGNED=0 step "$s" 400 python bench/rccl_self_overhead.py --K 24 \
             --periodic "$d" --steps 320 --pattern opop --spacing equal --out "$OUT/$s.json" || exit 1 ;;
    eq_x_a3072|eq_y_a3072|eq_xy_a3072) d=${s#eq_}; d=${d%_a3072}
             RMA_FRAME_ALIGNED=1 step "$s" 400 python bench/rccl_self_overhead.py --K 24 \
             --periodic "$d" --steps 320 --pattern opop --spacing equal --chunk2 3072 \
             --out "$OUT/$s.json" || exit 1 ;;
    eq16k_x|eq16k_y|eq16k_xy) d=${s#eq16k_}
             step "$s" 300 python bench/rccl_self_overhead.py --n 16384 --K 24 --periodic "$d" \
             --steps 960 --pattern opop --spacing equal --out "$OUT/$s.json" || exit 1 ;;
    eqn*) # eqn<N>_<dims>[_strips][_cd<D>][_bol|_btask]: N^2 tile, K=24, equal coefficients
             t=${s#eqn}; n=${t%%_*}; t=${t#*_}; d=${t%%_*}; fa=""; cd=""; fb=""; hm=""; lg=""
             mc=""; pp=""; sk=""; va="perf_hide"; fu=""; fd=""
             for tok in ${t//_/ }; do case $tok in strips) fa=0 ;; cd*) cd=${tok#cd} ;;
               skip) sk=1 ;; perf) va=perf ;; fused) fu=1 ;; split) fu=0 ;; fd*) fd=${tok#fd} ;;
               bol) fb=ol ;; btask) fb=task ;; nomerge) hm=0 ;; nolag) lg=0 ;;
               ch*) mc=${tok#ch} ;; pp*) pp=${tok#pp} ;; esac; done
             RMA_EXEC_LAG=$lg RMA_HALO_MERGED=$hm RMA_FRAME_BANDS=$fb RMA_FRAME_CHUNK_DIV=$cd \
             RMA_FRAME_ALIGNED=$fa RMA_DIAG_SKIP_EXCHANGE=$sk RMA_EXEC_FUSED=$fu RMA_FUSED_FRAME_DIV=$fd \
             step "$s" 300 env \
             ${mc:+NCCL_MAX_P2P_NCHANNELS=$mc} ${pp:+NCCL_NCHANNELS_PER_PEER=$pp} \
             python bench/rccl_self_overhead.py --n "$n" --K 24 --variants $va \
             --periodic "$d" --steps 2400 --pattern opop --spacing equal --out "$OUT/$s.json" || exit 1 ;;
    tests_fused) step tests_fused 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
             "tests/test_multirank_gpu.py::test_fused_frame_first_passes_bitwise" \
             "tests/test_multirank_gpu.py::test_fused_passes_over_rccl_self_equal_the_split_passes" \
             "tests/test_multirank_gpu.py::test_fused_pass_wait_timeout_is_reported_not_hung" \
             "tests/test_capi_gpu.py::test_capi_fused_passes_checked_and_bitwise" \
             "tests/test_multirank_gpu.py::test_fused_one_step_passes_bitwise" \
             "tests/test_multirank_gpu.py::test_fused_one_step_passes_over_rccl_self_equal_split" \
             -p no:cacheprovider || exit 1 ;;
    eq_xy_fused|eq_xy_split) fu=1; [ $s = eq_xy_split ] && fu=0
             RMA_EXEC_FUSED=$fu step "$s" 400 python bench/rccl_self_overhead.py --K 24 --periodic xy \
             --steps 320 --pattern opop --spacing equal --out "$OUT/$s.json" || exit 1 ;;
    eqauto2) for t in eqn4096_xy eqn5120_xy eqn6144_xy eqn7168_xy eqn8192_xy eqn2048_xy eqn4096_x \
                      eqn4096_y eqn6144_x eqn6144_y; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    eqy) for t in eqn6144_y_split eqn6144_y_fused eqn6144_y_split eqn6144_y_fused eqn5120_y_split \
                  eqn5120_y_fused eqn6144_x_split eqn6144_x_fused; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    trace_fused) prof trace_fused 300 --kernel-trace -d "$R/$OUT/trace_fused" -o run -- python3 \
             "$R/bench/rccl_self_overhead.py" --n 8192 --K 24 --periodic xy --steps 240 --pattern p \
             --spacing equal --out "$R/$OUT/trace_fused.json" || exit 1 ;;
    trace_fused_y) RMA_EXEC_FUSED=1 prof trace_fused_y 300 --kernel-trace -d "$R/$OUT/trace_fused_y" -o run \
             -- python3 "$R/bench/rccl_self_overhead.py" --n 6144 --K 24 --periodic y --steps 240 \
             --pattern op --spacing equal --out "$R/$OUT/trace_fused_y.json" || exit 1 ;;
    k1fused) for n in 8192 12288 16384 4096; do
               for fs in 0 1; do
                 RMA_EXEC_FUSED_STEP=$fs step "k1_${n}_fs$fs" 300 python bench/rccl_self_overhead.py --n $n \
                   --K 1 --variants perf_hide --periodic xy --steps 400 --pattern opop --spacing equal \
                   --out "$OUT/k1_${n}_fs$fs.json" || exit 1
               done
             done ;;
    eqbound) for t in eqn6144_xy_split eqn6144_xy_fused eqn7168_xy_split eqn7168_xy_fused \
                      eqn5120_xy_split eqn5120_xy_fused eqn8192_y_split eqn8192_y_fused; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    eqfdiv) for t in eqn2048_xy_split eqn2048_xy_fused eqn2048_xy_fused_fd2 eqn2048_xy_fused_fd3 \
                     eqn4096_xy_split eqn4096_xy_fused_fd2 eqn4096_xy_fused_fd4 eqn8192_xy_fused \
                     eqn8192_xy_fused_fd2; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    eqauto) for t in eq_xy_split eq_xy_fused eqn12288_xy_split eqn12288_xy_fused eqn12288_xy \
                     eqn8192_xy eqn4096_xy eqn2048_xy; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    eqfused) for t in eqn8192_xy eqn8192_xy_fused eqn2048_xy eqn2048_xy_fused eqn4096_xy \
                      eqn4096_xy_fused eqn16384_xy eqn16384_xy_fused eqn8192_x eqn8192_x_fused \
                      eqn8192_y eqn8192_y_fused; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    k1tiles) for n in 4096 8192 12288 16384; do
               step "k1_$n" 300 python bench/rccl_self_overhead.py --n $n --K 1 --variants perf_hide,perf \
                 --periodic xy --steps 400 --pattern opop --spacing equal --out "$OUT/k1_$n.json" || exit 1
             done ;;
    eqsplit) for t in eqn8192_xy eqn8192_xy_skip eqn8192_xy_perf eqn2048_xy eqn2048_xy_skip \
                      eqn2048_xy_perf eqn4096_xy eqn4096_xy_skip; do
               bash "$0" OUT="$OUT" "$t" || exit 1; done ;;
    chunk_sweep) step chunk_sweep 400 python bench/pass_sweep.py --pipe 20,24 --pipec "" \
             --ldsdpp "" --old "" --alt "" --rounds 3 \
             --chunks "20:2048/3072/4096/6144,24:2048/3072/4096/6144" \
             --out "$OUT/chunk_sweep.json" || exit 1 ;;
    power_coef) step power_coef 400 python bench/power_probe.py --seconds 5 \
             --configs pipe:24:iso,pipe:24:aniso,pipe:24:pow2,pipe:24:iso,pipe:24:aniso,pipe:24:pow2 \
             --out "$OUT/power_coef.json" || exit 1 ;;
    coef_ry) step coef_ry 400 python bench/rccl_self_overhead.py --K 24 --periodic x --steps 320 \
             --pattern oo --spacing anisotropic --variants perf --out "$OUT/coef_ry.json" || exit 1 ;;
    host4096|host2048) n=${s#host}
             step "$s" 300 python bench/rccl_self_overhead.py --n "$n" --K 1 --variants perf_hide \
             --steps 400 --pattern opop --out "$OUT/$s.json" || exit 1 ;;
    shape_alt) step shape_alt 400 python bench/interior_shape_probe.py --K 24 --coef physics \
             --alternate 12 --reps 2 --rects open,owned_x,owned_y,owned_xy \
             --out "$OUT/shape_alt.json" || exit 1 ;;
    shape_alt_g) step shape_alt_g 400 python bench/interior_shape_probe.py --K 24 --coef physics \
             --init gaussian --alternate 12 --reps 2 --rects open,owned_x,owned_y,owned_xy \
             --out "$OUT/shape_alt_g.json" || exit 1 ;;
    shape_r3) step shape_r3 400 python bench/interior_shape_probe.py --K 24 --coef physics \
             --alternate 8 --reps 2 --rects open,al_x,band_y,hyb_xy,al1536_xy,hyb_xy_rowphase \
             --out "$OUT/shape_r3.json" || exit 1 ;;
    eq_xy_bandtask) RMA_FRAME_BANDS=task step eq_xy_bandtask 400 python bench/rccl_self_overhead.py \
             --K 24 --periodic xy --steps 320 --pattern opop --spacing equal \
             --out "$OUT/eq_xy_bandtask.json" || exit 1 ;;
    shape_alt_lowns) step shape_alt_lowns 400 python bench/interior_shape_probe.py --K 24 \
             --coef physics --alternate 12 --reps 2 --rects open,owned_x,owned_y,owned_xy \
             --nosync --stream low --out "$OUT/shape_alt_lowns.json" || exit 1 ;;
    nbr_x_plain) RMA_EXEC_STREAMS=plain step nbr_x_plain 400 python bench/rccl_self_overhead.py \
             --K 24 --periodic x --steps 320 --pattern opop --out "$OUT/nbr_x_plain.json" || exit 1 ;;
    nbr_x_perf) step nbr_x_perf 400 python bench/rccl_self_overhead.py --K 24 --periodic x \
             --variants perf --steps 320 --pattern opop --out "$OUT/nbr_x_perf.json" || exit 1 ;;
    pmc_x_perf_a) prof pmc_x_perf_a 240 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
             SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
             --output-format csv -d "$R/$OUT/pmc_x_perf_a" -o run -- python3 \
             "$R/bench/rccl_self_overhead.py" --K 24 --periodic x --variants perf --steps 96 \
             --pattern op || exit 1 ;;
    pmc_x_perf_b) prof pmc_x_perf_b 240 --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SALU \
             GRBM_COUNT --output-format csv -d "$R/$OUT/pmc_x_perf_b" -o run \
             -- python3 "$R/bench/rccl_self_overhead.py" --K 24 --periodic x --variants perf \
             --steps 96 --pattern op || exit 1 ;;
    rccl_capture) step rccl_capture 120 build/bench/rccl_capture_probe 1048576 0 || exit 1 ;;
    capi_graph) RMA_RCCL_GRAPH=1 RMA_RCCL_BLOCKING=1 step capi_graph 180 \
             build/examples/rccl_graph_capi 4096 400 1 || exit 1 ;;
    capi_graph_k24) RMA_RCCL_GRAPH=1 RMA_RCCL_BLOCKING=1 step capi_graph_k24 180 \
             build/examples/rccl_graph_capi 4096 2400 24 || exit 1 ;;
    rccl_graph) step rccl_graph 500 python bench/rccl_graph_probe.py --n 4096 --steps 400 \
             --out "$OUT/rccl_graph.json" || exit 1 ;;
    trace20) prof trace20 300 --kernel-trace --stats --output-format csv -d "$R/$OUT/trace20" \
             -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== all steps done"
