#!/bin/bash
# Two SQ counter passes (rocprofv3 --pmc, one run each) over a probe command.
# usage: tools/pmc_probe.sh TAG cmd...   -> gpurun_out/pmc_TAG_{a,b}/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=$1; shift
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM"
timeout -s KILL 120 rocprofv3 --pmc $A -f csv -d gpurun_out/pmc_${TAG}_a -o run -- "$@" > gpurun_out/pmc_${TAG}_a.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $B -f csv -d gpurun_out/pmc_${TAG}_b -o run -- "$@" > gpurun_out/pmc_${TAG}_b.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_b.log; exit 1; }
echo "pmc $TAG ok"
