set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/probe_embed.py --precision split --iters 3 > gpurun_out/probe_plain.log 2>&1 &&
timeout -k 10 120 python3 tools/probe_embed.py --precision split --iters 3 --phase > gpurun_out/probe_phase.log 2>&1 &&
bash tools/ablate_embed.sh
