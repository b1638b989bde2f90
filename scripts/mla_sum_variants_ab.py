"""A/B of the MFMA row sums (sum_mfma=False / True) on the paged and persistent MLA decode examples, through their mains."""
import sys
sys.path[:0] = ["examples/deepseek_mla"]
for modname, fn in (("example_mla_decode_paged", "mla_decode_paged"), ("example_mla_decode_persistent", "mla_decode_persistent")):
    m = __import__(modname)
    orig = getattr(m, fn)
    for sm in (False, True):
        setattr(m, fn, lambda *a, _o=orig, _sm=sm, **k: _o(*a, sum_mfma=_sm, **k))
        print(f"{modname} sum_mfma={sm}:", flush=True)
        m.main()
    setattr(m, fn, orig)
