for sh in 2,200,336,256,256,3,1 2,100,168,128,128,3,1 2,50,84,256,256,3,1 2,25,42,512,512,3,1 2,200,336,64,256,1,1 2,50,84,1024,256,1,1 2,50,84,256,1024,1,1; do
  timeout -k 5 60 python tools/conv_one.py --shape $sh --mode x3 --iters 20 || exit 1
  timeout -k 5 60 python tools/conv_one.py --shape $sh --mode split --iters 20 || exit 1
done
