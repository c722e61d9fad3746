#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/membench.py > gpurun_out/membench.json 2>gpurun_out/membench.err; c=$?; cat gpurun_out/membench.json; exit $c
