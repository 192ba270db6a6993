#!/bin/bash
# drop a database's collections and blobs (reference: remove_results.sh)
cd "$(dirname "$0")"
python -m lua_mapreduce_1_amd.cli.remove_results ${1:-127.0.0.1:27027} ${2:-wordcount}
