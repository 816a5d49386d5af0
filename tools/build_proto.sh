#!/bin/bash
# Builds the stream-structure prototypes (tools/proto_stream.hip) into tools/proto_bin/.
cd "$(dirname "$0")"
mk() { n=$1; shift; /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 "$@" proto_stream.hip -o proto_bin/$n 2>/dev/null || echo "FAIL $n"; }
mk a512  -DNT=512 -DTPW=1 -DNS=2 &
mk a512nobar -DNT=512 -DTPW=1 -DNS=2 -DBARRIER=0 -DDMA=0 &
mk a512ns4 -DNT=512 -DTPW=1 -DNS=4 &
mk a512nog -DNT=512 -DTPW=1 -DNS=2 -DGROUPS=0 &
mk b256t2 -DNT=256 -DTPW=2 -DNS=2 &
mk b256t2ns4 -DNT=256 -DTPW=2 -DNS=4 &
mk b256t2nobar -DNT=256 -DTPW=2 -DNS=2 -DBARRIER=0 -DDMA=0 &
mk b256t1ns4 -DNT=256 -DTPW=1 -DNS=4 &
mk b256t2ns4pd4 -DNT=256 -DTPW=2 -DNS=4 -DPD=4 &
mk b256t2ns4nog -DNT=256 -DTPW=2 -DNS=4 -DGROUPS=0 &
wait
