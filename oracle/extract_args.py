"""Read `llvm-readelf --notes` of the reference code object on stdin and print its
kernarg layout ("arg <offset>" per explicit argument in order, "<hidden kind>
<offset>" for hidden ones) for ref_launch.c.  Oracle build tooling only."""
import sys

import yaml


def main():
    text = sys.stdin.read()
    start = text.index("---")
    end = text.index("\n...", start)
    meta = yaml.safe_load(text[start:end])
    (kern,) = [k for k in meta["amdhsa.kernels"] if k[".name"] == "trace"]
    for a in kern[".args"]:
        kind = a[".value_kind"]
        if kind.startswith("hidden_"):
            print(kind, a[".offset"])
        else:
            print("arg", a[".offset"])
    print("# kernarg_segment_size", kern[".kernarg_segment_size"])
    print("# private_segment_fixed_size", kern[".private_segment_fixed_size"])


if __name__ == "__main__":
    main()
