set -o pipefail
A=or-gym-inventory_amd/invsim/_lib/ablate
bash tools/ab.sh invmgmt_backlog step cur $A/libinvsim_NO_WINDOW.so $A/libinvsim_NO_OBS.so $A/libinvsim_NO_POISSON.so
