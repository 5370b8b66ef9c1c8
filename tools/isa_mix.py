#!/usr/bin/env python3
"""Static instruction mix of the render kernels in a gfx950 assembly file
(hipcc --offload-device-only -S): per kernel, VALU count and the classes the
exact/fast A/Bs act on (divisions, square roots, selects, compares, min/max).

    python tools/isa_mix.py /tmp/exact.s [name-substring]
"""
import re
import sys
from collections import Counter


def kernels(text):
    cur, body = None, []
    for line in text.splitlines():
        m = re.match(r"^(_Z\w+):", line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur and line.startswith("\t") and not line.strip().startswith((".", ";")):
            body.append(line.strip().split()[0])
        elif cur and line.startswith(".Lfunc_end"):
            yield cur, body
            cur, body = None, []


def main():
    text = open(sys.argv[1]).read()
    pat = sys.argv[2] if len(sys.argv) > 2 else "render"
    for name, ins in kernels(text):
        if pat not in name:
            continue
        c = Counter(ins)
        g = lambda pre: sum(v for k, v in c.items() if k.startswith(pre))  # noqa: E731
        print(f"{name[:100]}\n  total {len(ins)} valu {g('v_')} salu {g('s_')} "
              f"div_scale {c['v_div_scale_f32']} rcp {g('v_rcp_f32')} rsq {g('v_rsq_f32')} "
              f"sqrt {g('v_sqrt_f32')} cndmask {g('v_cndmask')} cmp {g('v_cmp')} "
              f"min {g('v_min')} max {g('v_max')} fma {g('v_fma') + g('v_fmac')} "
              f"mul {g('v_mul_f32')} add {g('v_add_f32') + g('v_sub_f32') + g('v_subrev_f32')} "
              f"f64 {sum(v for k, v in c.items() if k.endswith('_f64'))}")


if __name__ == "__main__":
    main()
