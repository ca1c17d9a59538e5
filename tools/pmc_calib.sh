# rocprofv3 counter calibration on known byte counts (tools/pmc_calib.py):
#   gpurun -- bash tools/pmc_calib.sh r05
# one --pmc run per counter set (rocprofv3 does not split them), then the
# summary into profiles/<round>/pmc_calibration.json
set -euo pipefail
R=${1:-r05}
OUT=gpurun_out/calib_$R
mkdir -p "$OUT" "profiles/$R"
export TMPDIR=/tmp
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 tools/pmc_calib.py run > "$OUT/$name.log" 2>&1
  cp "$(find "$OUT/$name" -name run_counter_collection.csv -print -quit)" "$OUT/$name.csv"
  rm -rf "${OUT:?}/$name"
}
pass rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass wrreq TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
python3 tools/pmc_calib.py summarize "profiles/$R/pmc_calibration.json" \
    "$OUT/rdreq.csv" "$OUT/fetch.csv" "$OUT/write.csv" "$OUT/wrreq.csv" > "$OUT/summary.txt"
cp "profiles/$R/pmc_calibration.json" "$OUT/"
