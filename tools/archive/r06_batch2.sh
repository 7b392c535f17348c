bash tools/r06_wrap.sh && bash tools/r06_chaintrace.sh
