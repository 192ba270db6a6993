#!/bin/bash
# WordCount example worker (reference: execute_example_worker.sh)
cd "$(dirname "$0")"
python execute_worker.py 127.0.0.1:27027 wordcount --max-iter 5 --quiet
