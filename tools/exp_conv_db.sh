#!/bin/bash
# DB (double-buffered LDS, 1 WG/CU) vs single-buffered (2 WGs/CU) per shape and mode.
# usage: tools/exp_conv_db.sh mode shape...
mode=$1; shift
for sh in "$@"; do
 for db in 0 1; do
  D2MI_CONV_DB=$db timeout -k 5 60 python tools/conv_one.py --shape $sh --mode $mode --iters 20 | sed "s/^/db=$db /" || exit 1
 done
done
