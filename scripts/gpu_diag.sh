# Localise a parity failure: each mode combination in its own process with its own time limit; stops at a crash.
mkdir -p gpurun_out
for c in "e2e 0 1" "e2e 1 1" "e2e 0 0" "unit 0 1" "unit 0 0"; do
  timeout -k 10 150 python -u scripts/diag_modes.py $c >> gpurun_out/diag.log 2>&1
  rc=$?
  echo "[$c] rc=$rc" >> gpurun_out/diag.log
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; break ;; esac
done
cat gpurun_out/diag.log | grep -v Warning
