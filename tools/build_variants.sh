# Kernel A/B experiments: rebuilds one source file with extra -D flags and links it with the
# other objects of the main build into var/<name>/librpst.so (select at run time with
# RPST_LIB=var/<name>/librpst.so). Usage, from the repo root after `make -C .../csrc`:
#   bash tools/build_variants.sh rpst_wino4.hip "a:-DRPST_W4_HW=0" "b:-DRPST_W4_HP=2" ...
set -e
SRC=$1; shift
C=rp-style-transfer_amd/csrc
OBJ=build/${SRC%.hip}.o
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function"
case $SRC in rpst_wino4.hip|rpst_wino4q.hip) FLAGS="$FLAGS -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form=1";; rpst_flash.hip) FLAGS="$FLAGS -mllvm -amdgpu-mfma-vgpr-form=1";; esac
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  mkdir -p var/$name
  /opt/rocm/bin/hipcc $FLAGS $defs -c $C/$SRC -o var/$name/${SRC%.hip}.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  objs=$(ls $C/build/*.o | grep -v "/${SRC%.hip}.o$")
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o var/$name/librpst.so $objs var/$name/${SRC%.hip}.o
  echo "var/$name/librpst.so"
done
