bash tools/r06_wrap.sh && bash tools/r06_perm.sh
