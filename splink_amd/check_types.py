"""`@check_types`: isinstance checks of annotated arguments (reference: splink/check_types.py:20-52).

The reference annotates Spark types; here the frame annotations accept pandas / pyarrow
inputs and the device-resident frames of splink_amd.frames, and a `spark` argument may be a
SparkSession, an AmdSession, None or the 'supress_warnings' test marker.
"""
from functools import wraps
from typing import Union, get_type_hints


def _possible_types(hint):
    origin = getattr(hint, "__origin__", None)
    if origin is Union:
        return hint.__args__
    return (hint,)


def check_types(func):
    hints = None

    @wraps(func)
    def wrapper(*args, **kwargs):
        nonlocal hints
        if hints is None:
            hints = get_type_hints(func)
        names = func.__code__.co_varnames[: func.__code__.co_argcount]
        bound = {**dict(zip(names, args)), **kwargs}
        for key, hint in hints.items():
            if key not in bound or key == "return":
                continue
            types = _possible_types(hint)
            if any(t is object for t in types):
                continue
            value = bound[key]
            if not isinstance(value, types):
                allowed = " or ".join(str(t) for t in types)
                raise TypeError(f"You passed the wrong type for argument {key}. "
                                f"You passed the argument {value} of type {type(value)}. "
                                f"The type for this argument should be {allowed}. ")
        return func(*args, **kwargs)

    return wrapper
