# PMC passes on the multi-step kernels (counters only with --kernel-trace-free
# --pmc runs; never combined with sys/runtime traces)
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/m
export HSA_ENABLE_IPC_MODE_LEGACY=0 RMA_PROBE_SET=tbk RMA_PROBE_REPS=2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/m/counters.txt 2>&1; echo "list rc=$?"
grep -oE "^\s*(SQ|TCP|TCC|TA|GRBM)[A-Z0-9_]*" $R/gpurun_out/m/counters.txt | sort -u | head -400 > $R/gpurun_out/m/counter_names.txt
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU_FP64 SQ_WAVES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/m/p$i -o run -- python3 $R/bench/pmc_probe.py > $R/gpurun_out/m/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
