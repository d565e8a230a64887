#!/bin/bash
# Python-side A/B: variants/tree_NAME = bench.py + the package + oracle at git revision REV (run with
# TDE_LIBRARY pointing at the current libtde.so; scripts/ab_trees.sh).
#   bash scripts/mk_tree_variant.sh NAME REV
set -eu
cd "$(dirname "$0")/.."
d=variants/tree_$1
rm -rf "$d"; mkdir -p "$d"
git archive "$2" bench.py tf_depth_estimation_amd oracle | tar -x -C "$d" --exclude='*.hip' --exclude='*.h' --exclude='*.cpp' --exclude='Makefile'
echo "$d <- $2"
