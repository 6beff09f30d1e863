# Round 6: where the rules trajectory's time goes, by instruction -- rocprofv3
# PC sampling of the driver's c3 command (attribute the
# rules' VALU by phase).  Stochastic (hardware) sampling first; host-trap
# sampling if this ROCm / box refuses the stochastic method with an ordinary
# error.  tools/pc_attrib.py maps the samples onto the code object's
# disassembly (basic blocks -> phases).
set -u
. tools/gpu_calls/attempt.sh r06i
R=$(pwd)
cd /tmp
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $R/$D/list_avail.txt 2>&1 || true
run() {
  timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method "$1" --pc-sampling-unit "$2" \
    --pc-sampling-interval "$3" --kernel-trace --output-format csv -d "$R/$D/pcs_$1" -o run \
    -- python3 "$R/bench.py" --config c3 --steps 40 --warmup 5 --no-cpu-baseline > "$R/$D/pcs_$1.log" 2>&1
}
run stochastic cycles 65536
rc=$?
echo "stochastic rc=$rc"
if [ $rc -ne 0 ]; then
  case $rc in 124|134|137|139) exit $rc ;; esac
  run host_trap time 50
  echo "host_trap rc=$?"
fi
cd "$R"
ls -laR "$D" | head -40
