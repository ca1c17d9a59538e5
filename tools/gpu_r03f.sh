# round 3: fp32 2-D GEMM N-fastest XCD order A/B; bf16 forward DMA GEMM XCD-contiguous order A/B (time + conv6 fwd traffic),
# and the f16x2 GEMM's SQ counters (conv6 shape)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03f
mkdir -p $OUT
for i in 1 2; do
  for x in 0 1; do
    NSM_F32_XCD2D=$x timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline --detail $OUT/bd_f32x${x}_$i.json > $OUT/b_f32x${x}_$i.log 2>&1 || exit $?
  done
done
for i in 1 2; do
  for x in 2 3; do
    NSM_BF16_XCD=$x timeout -k 10 200 python bench.py --dtype bf16 --batch 64 --steps 10 --warmup 3 --no-secondary --no-cpu-baseline --detail $OUT/bd_x${x}_$i.json > $OUT/b_x${x}_$i.log 2>&1 || exit $?
  done
done
for x in 2 3; do
  NSM_BF16_XCD=$x NSM_STAGE_MARKS=1 timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $OUT/rd_x$x -o run -- python3 bench.py --dtype bf16 --batch 64 --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $OUT/prd_x$x.log 2>&1 || exit $?
  NSM_BF16_XCD=$x NSM_STAGE_MARKS=1 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/wr_x$x -o run -- python3 bench.py --dtype bf16 --batch 64 --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $OUT/pwr_x$x.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py bf16 $OUT/traffic_bf16_x$x.json $(find $OUT/rd_x$x -name run_counter_collection.csv) $(find $OUT/wr_x$x -name run_counter_collection.csv) > /dev/null
  rm -rf $OUT/rd_x$x $OUT/wr_x$x
done
SHAPES=0 REPS=50 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq16 -o run -- python3 tools/bench_split16.py > $OUT/sq16.log 2>&1 || exit $?
cp $(find $OUT/sq16 -name run_counter_collection.csv) $OUT/sq16.csv; rm -rf $OUT/sq16
