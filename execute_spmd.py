#!/usr/bin/env python
"""Repository-root shortcut for lua_mapreduce_1_amd.cli.execute_spmd (SPMD form of execute_server.lua)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lua_mapreduce_1_amd.cli.execute_spmd import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
