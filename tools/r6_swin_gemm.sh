#!/bin/bash
# Video Swin stage GEMM shapes (config 5) under the forced GEMM variants given as arguments
set -o pipefail
export DSVT_CUSTOM="s3qkv:3136:1152:384:0,s3fc1:3136:1536:384:1,s3fc2:3136:384:1536:2,s3proj:3136:384:384:2,s4qkv:784:2304:768:0,s4fc1:784:3072:768:1,s4fc2:784:768:3072:2,s4proj:784:768:768:2,s2qkv:12544:576:192:0,s2fc1:12544:768:192:1,s2fc2:12544:192:768:2,s2proj:12544:192:192:2,s1qkv:50176:288:128:0,s1fc1:50176:384:128:1,s1fc2:50176:96:384:2,s1proj:50176:96:128:2,mrg3:784:768:1536:2,mrg2:3136:384:768:2"
export DSVT_SHAPES="s3qkv,s3fc1,s3fc2,s3proj,s4qkv,s4fc1,s4fc2,s4proj,s2qkv,s2fc1,s2fc2,s2proj,s1qkv,s1fc1,s1fc2,s1proj,mrg3,mrg2"
timeout -k 10 300 python -u tools/gemm_bench.py "$@"
