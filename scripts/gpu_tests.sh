#!/bin/bash
# GPU parity tests for the given test files (default: all @gpu tests), one process, each
# test under a thread timeout; the log goes to gpurun_out/t.log and its tail to stdout.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?
tail -15 gpurun_out/t.log
exit $rc
