A=or-gym-inventory_amd/invsim/_lib/ablate
bash tools/ab.sh newsvendor step cur $A/libinvsim_LA_NOMULT.so $A/libinvsim_LA_NOPTRS.so
