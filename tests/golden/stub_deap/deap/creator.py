"""deap.creator layout stand-in: classes are made in this module's namespace."""


def create(name, base, **kargs):
    per_instance = {k: v for k, v in kargs.items() if isinstance(v, type)}
    cls_attrs = {k: v for k, v in kargs.items() if not isinstance(v, type)}

    def __init__(self, *args, **kw):
        for k, v in per_instance.items():
            setattr(self, k, v())
        base.__init__(self, *args, **kw)

    cls = type(str(name), (base,), cls_attrs)
    cls.__init__ = __init__
    globals()[name] = cls
