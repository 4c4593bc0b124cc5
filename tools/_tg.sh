#!/bin/bash
# tile-order sweep for the 256x256 kernel (diagnostic)
for g in 0 4 8 16 32; do
  echo "== DSVT_TILE_GROUP=$g"
  DSVT_SHAPES=qkv_g,fc1_g,proj_g,qkv_l,fc1_l DSVT_TILE_GROUP=$g timeout -k 10 120 python -u tools/gemm_bench.py 10 20 || exit 1
done
