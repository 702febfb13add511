cd $GRAFT_REPO_ROOT
timeout -k 10 200 python scripts/diag_vae_race2.py base 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python scripts/diag_vae_race2.py foreach_zero 2>&1 | grep -v amdgpu.ids
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python scripts/diag_vae_race2.py base 2>&1 | grep -v amdgpu.ids
