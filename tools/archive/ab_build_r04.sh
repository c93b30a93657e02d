#!/bin/bash
# The round-4 build (2ba43e1) next to this tree, for the cfg-2 class-scan A/B
# (tools/exp_class_ab.py): its library sources and Python package only,
# built here into ab/r04/ (git-ignored; it travels to the GPU box with the
# tree like the product's own .so).
set -e
rm -rf ab/r04 && mkdir -p ab/r04
git archive 2ba43e1 vectorscan_amd include oracle Makefile tests/c tools/dropin_threads.c | tar -x -C ab/r04
make -C ab/r04 -j8 all
