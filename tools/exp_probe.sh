#!/bin/bash
set -e
OUT=gpurun_out/probe
mkdir -p $OUT
timeout -k 10 120 ./tools/probe_stream > $OUT/probe.txt 2>&1
