#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/ab_smallk.py default,build/variants/libbcmpc_old47.so,build/variants/libbcmpc_vB.so,build/variants/libbcmpc_vD.so "runsh_noln cfg1" > gpurun_out/r03_ab_team2.txt 2>&1
