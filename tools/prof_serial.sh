# Serialised step timelines (the bench's last attribution step: weight
# gradients on the main stream) of the fp32 B=8 and bf16 B=64 steps
set -euo pipefail
mkdir -p gpurun_out/ser
bash tools/prof_step.sh
cp gpurun_out/prof_step/timeline.txt gpurun_out/ser/step_b8_f32.txt
CFG="--dtype bf16 --batch 64" bash tools/prof_step.sh
cp gpurun_out/prof_step/timeline.txt gpurun_out/ser/step_b64_bf16.txt
