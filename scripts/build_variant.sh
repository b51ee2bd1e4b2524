# Build a variant of libpqp with extra -D flags on one source file, for A/B
# timing in one process (PQP_LIB=ab/libpqp_NAME.so).  Run here, on the CPU:
#   bash scripts/build_variant.sh NAME SOURCE "-DX=1 -DY=2"
set -e
cd "$(dirname "$0")/../pqp-for-mpc_amd"
NAME=$1; SRC=$2; DEFS=$3
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -Wall -Wno-unused-result"
mkdir -p ../ab build/ab_$NAME
/opt/rocm/bin/hipcc $HIPFLAGS $DEFS -c csrc/$SRC.hip -o build/ab_$NAME/$SRC.o
OBJS=""
for o in build/pqp_kernels.o build/pqp_tiny.o build/pqp_wide.o build/pqp_persist.o build/pqp_converge.o build/pqp_capi.o build/pqp_host.o build/pqp_io.o; do
  b=$(basename $o .o)
  if [ "$b" = "$SRC" ]; then OBJS="$OBJS build/ab_$NAME/$SRC.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc $HIPFLAGS -shared $OBJS -o ../ab/libpqp_$NAME.so
echo ab/libpqp_$NAME.so
