#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 150 python -u tools/adam_prof.py 512 100000 512 300 > gpurun_out/adamprof_${1:-x}.txt 2>&1
