# r6: r6q (RetinaNet post variants) then r6p (split B[R] tests + A/B bench)
bash tools/gpu/r6q.sh && bash tools/gpu/r6p.sh
