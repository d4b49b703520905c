PT_LIBDIR=$GRAFT_REPO_ROOT/pathtracerwithcuda_amd/lib_seg timeout -k 10 200 python tools/uprof.py
