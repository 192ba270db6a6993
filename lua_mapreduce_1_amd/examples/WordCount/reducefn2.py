"""WordCount general reducer (reference: examples/WordCount/reducefn2.lua):
same sum, no reducer flags (every key goes through reducefn)."""


def init(arg):
    pass


def reducefn(key, values, emit):
    emit(sum(values))


combinerfn = reducefn
