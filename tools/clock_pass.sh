# rocprofv3 MFMA-busy / clock pass over tools/clock_probe.py (long dispatches: the clock under sustained
# MFMA load), condensed to gpurun_out/clock_pass.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --output-format rocpd --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
  -d gpurun_out/clk -o run -- python3 tools/clock_probe.py > gpurun_out/clock_probe.log 2>&1 || exit 1
python3 - <<'PY'
import glob, json, sys
sys.path.insert(0, "tools")
import rocpd_summary as r
db = glob.glob("gpurun_out/clk/**/*results.db", recursive=True)[0]
out = {k: v for k, v in r.sq_pass(db).items() if "gemm" in k}
json.dump(out, open("gpurun_out/clock_pass.json", "w"), indent=1)
for k, v in out.items():
    print(k, v.get("launches"), round(v["avg_ns"] / 1e6, 2), "ms", v.get("eff_clock_ghz"), v.get("mfma_busy_frac"), v.get("mfma_busy_of_peak"))
PY
rm -rf gpurun_out/clk
