"""WordCount finalfn (reference: examples/WordCount/finalfn.lua): print
``count key`` and return True (remove the result files)."""


def init(arg):
    pass


def finalfn(pairs_iterator):
    for key, values in pairs_iterator:
        print(values[0], key)
    return True
