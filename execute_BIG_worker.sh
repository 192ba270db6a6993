#!/bin/bash
# WordCountBig worker (reference: execute_BIG_worker.sh)
cd "$(dirname "$0")"
python execute_worker.py 127.0.0.1:27027 wordcountBIG --max-iter 5
