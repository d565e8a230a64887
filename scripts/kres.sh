#!/bin/bash
# Register / LDS / occupancy table of the conv kernel instantiations (diagnostic):  bash scripts/kres.sh [file.hip]
F=${1:-tf_depth_estimation_amd/csrc/conv_igemm.hip}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c "$F" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed 's/.*remark: //; s/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name/ {name=$3} /^ *VGPRs:/ {v=$2} /AGPRs:/ {a=$2} /VGPRs Spill/ {sp=$3} /Occupancy/ {o=$3} /LDS Size/ {l=$4; print name, "vgpr", v, "agpr", a, "spill", sp, "occ", o, "lds", l}' |
  c++filt | sed 's/(anonymous namespace):://g; s/void //; s/(ConvArgs)//'
