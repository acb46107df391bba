#!/bin/bash
# Build ablated copies of libmarlsat.so into ab/<tag>.so (timing diagnostics only: the ablated
# kernels compute wrong results).  usage: bash profiles/build_abl.sh <tag> <file.hip> <-Dflags...>
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; SRC=$2; shift 2
mkdir -p /tmp/abobj_$TAG $R/ab
make -s -C $R/marl-sat_amd >/dev/null
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -I$R/include -I$R/marl-sat_amd/csrc"
/opt/rocm/bin/hipcc $FLAGS "$@" -c $R/marl-sat_amd/csrc/$SRC -o /tmp/abobj_$TAG/${SRC%.hip}.o
OBJS=""
for o in $R/marl-sat_amd/build/*.o; do
  b=$(basename $o)
  [ "$b" = debug.o ] && continue
  if [ "$b" = "${SRC%.hip}.o" ]; then OBJS="$OBJS /tmp/abobj_$TAG/$b"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/ab/$TAG.so $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $R/ab/$TAG.so
