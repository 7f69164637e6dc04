set -o pipefail
A=or-gym-inventory_amd/invsim/_lib/ablate
bash tools/ab.sh newsvendor rollout cur $A/libinvsim_ROLL_NO_MULT.so $A/libinvsim_ROLL_NO_PTRS.so $A/libinvsim_ROLL_NO_DRAW.so $A/libinvsim_ROLL_NO_STORE.so
