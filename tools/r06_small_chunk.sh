#!/bin/bash
# round 6: small launches (one tile of one sample, the reference's Graphics::Render call; C1's
# 256x256 frame) with smaller work claims spread over every CU, against one 128-unit chunk per wave
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python tools/abrun.py --cases c2t,rm3t,c3t,c1 --rounds 20 off="env:RMR_SMALL_CHUNK=0" c64="env:RMR_SMALL_CHUNK=64" c32="env:RMR_SMALL_CHUNK=32" c16="env:RMR_SMALL_CHUNK=16" c8="env:RMR_SMALL_CHUNK=8" > $O/r06m_small_chunk.log 2>&1 || exit $?
timeout -k 10 300 python tools/abrun.py --cases c2,c4 --rounds 2 off="env:RMR_SMALL_CHUNK=0" c32="env:RMR_SMALL_CHUNK=32" >> $O/r06m_small_chunk.log 2>&1 || exit $?
grep '"case"' $O/r06m_small_chunk.log | cut -c1-3000
