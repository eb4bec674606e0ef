set -e
mkdir -p gpurun_out/pool
rm -f gpurun_out/pool/sweep.jsonl
CONFIG=C3 SPP=256 scripts/extend_sweep.sh gpurun_out/pool/sweep.jsonl "C=C3" "OCTPT_POOL=536870912,C=C3" "C=C3" "OCTPT_POOL=536870912,C=C3"
CONFIG=C4 SPP=64 scripts/extend_sweep.sh gpurun_out/pool/sweep.jsonl "C=C4" "OCTPT_POOL=536870912,C=C4"
