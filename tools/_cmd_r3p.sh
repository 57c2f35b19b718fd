for n in 256 512 1024; do for k in 0 3; do OCRK_CTC_NT=$n OCRK_CTC_SKIP=$k timeout -k 10 60 python -u tools/bench_ctc.py 2>&1 | grep "LDS=1" | sed "s/^/nt=$n skip=$k /"; done; done
