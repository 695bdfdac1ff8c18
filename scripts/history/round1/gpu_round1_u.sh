# sweep at the 288 GB tile + PMC of the overlapped-strip K-step kernels
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/u
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench/stencil_sweep.py --n 101376 --rounds 3 --iters 2 --chunks 4 --unrolls 4 --nts 3 --xcds 1 --no-roof --tbk 4,6,8 --tbk-chunks 128,256,512,1024 --tbk-xcds 1 --tbk-vecs 2 --out gpurun_out/u/sweep_tbk_101k.json > gpurun_out/u/sweep.log 2>&1
rc=$?; grep -E '"best' gpurun_out/u/sweep.log; case $rc in 0) ;; *) exit $rc;; esac
export RMA_PROBE_SET=tbk RMA_PROBE_REPS=2
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU_FP64 SQ_WAVES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/u/p$i -o run -- python3 $R/bench/pmc_probe.py > $R/gpurun_out/u/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/u/trace -o run -- python3 bench.py --steps 120 --single-step-steps 24 > gpurun_out/u/trace_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 gpurun_out/u/trace_bench.log | cut -c1-200; exit $rc
