cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for a in "0 0" "0 1" "1 0" "1 1"; do
  echo "== probe $a"; timeout -k 10 120 python scripts/rccl_probe.py $a > gpurun_out/probe.log 2>&1; rc=$?; tail -3 gpurun_out/probe.log; echo "rc=$rc"
  case $rc in 124|137) echo "timeout, stop"; exit $rc;; esac
done
