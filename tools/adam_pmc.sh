#!/bin/bash
# SQ counters of the persistent Adam kernel at C3 (one pass; <= 8 SQ counters).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d $R/gpurun_out/adam_pmc -o adam_pmc --output-format csv -- python3 $R/tools/adam_prof.py 512 100000 512 300
