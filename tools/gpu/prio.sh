A=or-gym-inventory_amd/invsim/_lib/ablate
bash tools/ab.sh newsvendor step cur $A/libinvsim_PRIO1.so $A/libinvsim_PRIO3.so
bash tools/ab.sh invmgmt_backlog step cur $A/libinvsim_PRIO1.so $A/libinvsim_PRIO3.so
