for sh in 256,14,14,256,256,3,1 2,200,336,256,256,3,1 2,100,168,256,256,3,1 2,50,84,256,256,3,1 2,100,168,128,128,3,1 2,25,42,512,512,3,1; do
  timeout -k 5 60 python tools/conv_one.py --shape $sh --mode split --iters 20 | sed "s/^/presplit /" || exit 1
  D2MI_CONV_PRESPLIT=0 timeout -k 5 60 python tools/conv_one.py --shape $sh --mode split --iters 20 | sed "s/^/staging  /" || exit 1
done
