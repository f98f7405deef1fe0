#!/bin/bash
# A/B of two builds of libd2mi_hip.so on the Mask R-CNN conv shapes.
# usage: tools/ab_conv.sh <lib A> <lib B> [mode]
# (each shape runs under its own time limit; a failure ends the script)
A=$1; B=$2; mode=${3:-split}
shapes=${SHAPES:-"2,200,336,256,256,3,1 2,100,168,256,256,3,1 2,100,168,128,128,3,1 2,200,336,64,256,1,1 2,200,336,256,64,1,1 2,100,168,128,512,1,1 2,100,168,512,128,1,1 2,50,84,256,256,3,1 64,14,14,256,256,3,1"}
for sh in $shapes; do
  for lib in $A $B; do
    D2MI_LIB=$lib timeout -k 5 60 python tools/conv_one.py --shape $sh --mode $mode --iters 20 \
      | sed "s|^|$(basename $lib) |" || exit 1
  done
done
