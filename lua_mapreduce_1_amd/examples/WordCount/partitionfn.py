"""WordCount partitionfn (reference: examples/WordCount/partitionfn.lua):
FNV-1 of the key bytes mod NUM_REDUCERS, computed exactly in uint32 (the
reference's Lua-double arithmetic drops low bits)."""
NUM_REDUCERS = 15
FNV_PRIME = 16777619
OFFSET_BASIS = 2166136261
MAX = 2 ** 32


def init(arg):
    pass


def partitionfn(key):
    h = OFFSET_BASIS
    for c in key.encode("utf-8", "surrogateescape"):
        h = (h * FNV_PRIME) % MAX
        h ^= c
    return h % NUM_REDUCERS


device_partition = ("fnv1", NUM_REDUCERS)
