"""Generate trivy_amd/data/builtin_rules.json from the reference's rule DATA.

Dev-time only (reads /root/reference, which does not exist on the GPU box).
Sources:
  pkg/fanal/secret/builtin-rules.go:12-74   categories
  pkg/fanal/secret/builtin-rules.go:77-84   reusable pattern fragments
  pkg/fanal/secret/builtin-rules.go:101-849 the 87 builtin rules
  pkg/fanal/secret/builtin-allow-rules.go:3-65 the 12 builtin allow rules
  pkg/fanal/secret/scanner.go:66-68  MustCompileWithoutWordPrefix = startWord + "(" + re + ")"

The JSON holds the fully expanded Go regex strings (fmt.Sprintf and the
word-prefix wrapper evaluated), so both the product (C++) and the oracle
(Python) start from identical pattern text.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
import golit  # noqa: E402

REF = "/root/reference/pkg/fanal/secret"
OUT = os.path.join(os.path.dirname(__file__), "..", "trivy_amd", "data", "builtin_rules.json")


def evaluate(node, env):
    if isinstance(node, str) or node is None or isinstance(node, (int, bool)):
        return node
    if isinstance(node, tuple) and node[0] == "+":
        return evaluate(node[1], env) + evaluate(node[2], env)
    if isinstance(node, golit.Ident):
        return env[node.name]
    if isinstance(node, golit.Call):
        args = [evaluate(a, env) for a in node.args]
        if node.fn == "fmt.Sprintf":
            fmt, rest = args[0], list(args[1:])
            out, i = "", 0
            while i < len(fmt):
                if fmt[i] == "%" and fmt[i + 1] == "s":
                    out += rest.pop(0)
                    i += 2
                elif fmt[i] == "%" and fmt[i + 1] == "%":
                    out += "%"
                    i += 2
                else:
                    out += fmt[i]
                    i += 1
            assert not rest
            return out
        if node.fn == "MustCompileWithoutWordPrefix":
            return "%s(%s)" % (env["startWord"], args[0])
        if node.fn == "MustCompile":
            return args[0]
        raise ValueError("unsupported call %s" % node.fn)
    if isinstance(node, golit.Composite):
        if node.typ and node.typ.startswith("[]"):
            return [evaluate(x, env) for x in node.items]
    raise ValueError("cannot evaluate %r" % (node,))


def parse_consts(src):
    env = {}
    # categories: CategoryX = types.SecretRuleCategory("X")
    start = golit.find_block(src, "var (")
    end = src.index("\n)", start)
    for line in src[start:end].splitlines():
        line = line.strip()
        if "=" in line:
            name, rhs = [x.strip() for x in line.split("=", 1)]
            env[name] = golit.go_unquote(rhs[rhs.index('"'):rhs.rindex('"') + 1])
    start = golit.find_block(src, "const (")
    end = src.index("\n)", start)
    for line in src[start:end].splitlines():
        line = line.strip()
        if "=" in line and not line.startswith("//"):
            name, rhs = [x.strip() for x in line.split("=", 1)]
            env[name] = golit.parse_expr_at(rhs, 0)
    return env


def main():
    rules_src = open(os.path.join(REF, "builtin-rules.go")).read()
    allow_src = open(os.path.join(REF, "builtin-allow-rules.go")).read()
    env = parse_consts(rules_src)
    rules_node = golit.parse_expr_at(rules_src, golit.find_block(rules_src, "var builtinRules = "))
    rules = []
    for r in rules_node.items:
        k = r.keyed
        rules.append({
            "id": evaluate(k["ID"], env),
            "category": evaluate(k.get("Category", ""), env) or "",
            "title": evaluate(k.get("Title", ""), env) or "",
            "severity": evaluate(k.get("Severity", ""), env) or "",
            "regex": evaluate(k["Regex"], env),
            "secret_group_name": evaluate(k.get("SecretGroupName", ""), env) or "",
            "keywords": evaluate(k.get("Keywords"), env) or [],
        })
    allow_node = golit.parse_expr_at(allow_src, golit.find_block(allow_src, "var builtinAllowRules = "))
    allows = []
    for a in allow_node.items:
        k = a.keyed
        allows.append({
            "id": evaluate(k["ID"], env),
            "description": evaluate(k.get("Description", ""), env) or "",
            "regex": evaluate(k.get("Regex"), env),
            "path": evaluate(k.get("Path"), env),
        })
    doc = {
        "_source": "mmorel-35/trivy pkg/fanal/secret/builtin-rules.go:101-849, "
                   "builtin-allow-rules.go:3-65 (rule data, regexes fully expanded)",
        "rules": rules,
        "allow_rules": allows,
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1, ensure_ascii=False)
        f.write("\n")
    print("wrote %d rules, %d allow rules -> %s" % (len(rules), len(allows), OUT))


if __name__ == "__main__":
    main()
