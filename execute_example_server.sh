#!/bin/bash
# WordCount example server (reference: execute_example_server.sh); $1 = storage
cd "$(dirname "$0")"
python execute_server.py --sleep 1 127.0.0.1:27027 wordcount \
  lua_mapreduce_1_amd.examples.WordCount.taskfn lua_mapreduce_1_amd.examples.WordCount.mapfn \
  lua_mapreduce_1_amd.examples.WordCount.partitionfn lua_mapreduce_1_amd.examples.WordCount.reducefn \
  lua_mapreduce_1_amd.examples.WordCount.finalfn lua_mapreduce_1_amd.examples.WordCount.reducefn ${1:-gridfs}
