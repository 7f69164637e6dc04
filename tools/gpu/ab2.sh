bash tools/ab.sh invmgmt_backlog step cur INVSIM_IM_LA_LAST=1 tools/abl_np.so
