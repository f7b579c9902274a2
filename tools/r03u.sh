NGS_BUILD_TIMING=1 timeout -k 10 300 python3 -c "
import time, bench
t=time.time(); c=bench.Corpus(10_000_000, row_size=4, wide=True); print('corpus', round(time.time()-t,2), flush=True)
t=time.time(); h=bench.build_index(c, True, 0, gram=2); print('indexW total', round(time.time()-t,2), flush=True)
" 2>&1 | grep -v amdgpu
