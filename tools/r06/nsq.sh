#!/bin/bash
set -o pipefail
O=gpurun_out/r06_nsq; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u tools/r06/nsq_diag.py > $O/diag.txt 2>&1; rc=$?; cat $O/diag.txt | grep -v amdgpu.ids; exit $rc
