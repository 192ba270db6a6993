"""WordCount general reducer with its batched device form: reducefn2's sum
(no reducer flags, ``combinerfn = reducefn``) plus ``device_reducefn``, the
same fold over EVERY key's value list at once on the GPU (ops/segments.py,
csrc/hip/segments.hip).  Because the combiner is the reducer, the device
plane runs ``device_reducefn`` as the map-side combiner as well
(parallel/reducers.py; reference: examples/WordCount/reducefn2.lua,
job.lua:92-96,198-202,264-284)."""
from lua_mapreduce_1_amd.ops import segments as _seg


def init(arg):
    pass


def reducefn(key, values, emit):
    emit(sum(values))


combinerfn = reducefn


def device_reducefn(keys, off, val):
    return _seg.sum(off, val)
