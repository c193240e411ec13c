"""Nested-dict helper (reference: fedsim/utils/dict_ops.py:7)."""


def apply_on_dict(dict_obj, fn, return_as_dict=False, *args, **kwargs):
    """Call ``fn(key, value, *args, **kwargs)`` for every item; optionally collect
    the results in a dict keyed like the input."""
    if dict_obj is None:
        return None
    ans = {}
    for key, value in dict_obj.items():
        x = fn(key, value, *args, **kwargs)
        if return_as_dict:
            ans[key] = x
    return ans if return_as_dict else None
