"""Turn the reference's own tests for the secret path into JSON fixtures.

Dev-time only: reads /root/reference (absent on the GPU box) and writes
  tests/golden/scanner_cases.json   <- pkg/fanal/secret/scanner_test.go:22-1351
  tests/golden/analyzer_cases.json  <- pkg/fanal/analyzer/secret/secret_test.go:16-258
  tests/golden/integration_cases.json <- integration/testdata/secrets.json.golden
                                         (+ integration/repo_test.go:366-372)
and copies the input / config files those tests read (data, not source) into
tests/golden/{scanner,analyzer,integration}/.
Each case is {name, config, input, path, want}; `want` is a types.Secret in the
reference's JSON field names (pkg/fanal/types/secret.go:5-20, misconf.go:48-61).
"""
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tools"))
import golit  # noqa: E402
import gen_builtin_rules  # noqa: E402

REF = "/root/reference"


def line_json(c):
    k = c.keyed
    return {
        "Number": k.get("Number", 0),
        "Content": k.get("Content", ""),
        "IsCause": k.get("IsCause", False),
        "Annotation": k.get("Annotation", ""),
        "Truncated": k.get("Truncated", False),
        "Highlighted": k.get("Highlighted", ""),
        "FirstCause": k.get("FirstCause", False),
        "LastCause": k.get("LastCause", False),
    }


class Ctx:
    def __init__(self, env):
        self.env = env
        self.findings = {}

    def val(self, node):
        if isinstance(node, golit.Ident):
            n = node.name
            if n in self.findings:
                return self.findings[n]
            if n.startswith("secret.Category"):
                return self.env[n.split(".", 1)[1]]
            raise KeyError(n)
        if isinstance(node, golit.Call) and node.fn == "filepath.Join":
            return "/".join(self.val(a) for a in node.args)
        return node

    def finding(self, c):
        k = c.keyed
        code = k.get("Code")
        lines = []
        if code is not None:
            lines = [line_json(x) for x in code.get("Lines").items]
        return {
            "RuleID": self.val(k.get("RuleID", "")),
            "Category": self.val(k.get("Category", "")),
            "Severity": self.val(k.get("Severity", "")),
            "Title": self.val(k.get("Title", "")),
            "StartLine": k.get("StartLine", 0),
            "EndLine": k.get("EndLine", 0),
            "Code": {"Lines": lines},
            "Match": self.val(k.get("Match", "")),
        }

    def secret(self, c):
        if c is None:
            return {"FilePath": "", "Findings": []}
        k = c.keyed
        fl = k.get("Findings")
        finds = [] if fl is None else [self.val(x) for x in fl.items]
        return {"FilePath": self.val(k.get("FilePath", "")), "Findings": finds}


def collect_findings(ctx, src):
    i = 0
    while True:
        j = src.find(":= types.SecretFinding{", i)
        if j < 0:
            break
        name = src[src.rfind("\n", 0, j) + 1:j].strip()
        node = golit.parse_expr_at(src, j + len(":= "))
        ctx.findings[name] = ctx.finding(node)
        i = j + 1


def test_table(src, marker):
    i = src.index(marker)
    j = src.index("\n\t}{", i)
    return golit.parse_expr_at(src, j + len("\n\t}"))


def stored(name):
    """Fixture file name in the repo: *.pyc inputs are kept as *.pyc.data
    (repo snapshots sent to the GPU box drop Python caches, *.pyc included)."""
    return name + ".data" if name.endswith(".pyc") else name


def copy_data(names, srcdir, dstdir):
    os.makedirs(dstdir, exist_ok=True)
    for n in sorted(set(names)):
        if not n:
            continue
        s = os.path.join(srcdir, n)
        d = os.path.join(dstdir, stored(n))
        os.makedirs(os.path.dirname(d), exist_ok=True)
        shutil.copyfile(s, d)


def scanner_cases(env):
    base = os.path.join(REF, "pkg/fanal/secret")
    src = open(os.path.join(base, "scanner_test.go")).read()
    ctx = Ctx(env)
    collect_findings(ctx, src)
    table = test_table(src, "tests := []struct {")
    cases, files = [], []
    for item in table.items:
        k = item.keyed
        cfg, inp = ctx.val(k["configPath"]), ctx.val(k["inputFilePath"])
        cases.append({"name": k["name"], "config": cfg, "input": inp, "path": inp,
                      "want": ctx.secret(k["want"]),
                      "ref": "pkg/fanal/secret/scanner_test.go"})
        files += [cfg, inp]
    copy_data(files, base, os.path.join(HERE, "scanner"))
    return cases


def analyzer_cases(env):
    base = os.path.join(REF, "pkg/fanal/analyzer/secret")
    src = open(os.path.join(base, "secret_test.go")).read()
    ctx = Ctx(env)
    collect_findings(ctx, src)
    table = test_table(src, "tests := []struct {")
    cases, files = [], []
    for item in table.items:
        k = item.keyed
        want = k.get("want")
        secrets = []
        if want is not None:
            secrets = [ctx.secret(s) for s in want.get("Secrets").items]
        cases.append({"name": k["name"], "config": k.get("configPath", ""),
                      "input": stored(k["filePath"]), "path": k["filePath"], "dir": k.get("dir", ""),
                      "want": secrets, "ref": "pkg/fanal/analyzer/secret/secret_test.go:16-214"})
        files += [k.get("configPath", ""), k["filePath"]]
    # TestSecretRequire (:216-258)
    req_i = src.index("func TestSecretRequire")
    table = test_table(src[req_i:], "tests := []struct {")
    required = []
    for item in table.items:
        k = item.keyed
        required.append({"name": k["name"], "path": k["filePath"], "want": k["want"]})
        files.append(k["filePath"])
    files.append("testdata/skip-tests-config.yaml")
    copy_data(files, base, os.path.join(HERE, "analyzer"))
    return cases, required


def integration_cases():
    base = os.path.join(REF, "integration/testdata")
    golden = json.load(open(os.path.join(base, "secrets.json.golden")))
    cases = []
    for res in golden["Results"]:
        if res.get("Class") != "secret":
            continue
        finds = []
        for s in res["Secrets"]:
            f = {k: s[k] for k in ("RuleID", "Category", "Severity", "Title",
                                   "StartLine", "EndLine", "Match")}
            f["Code"] = {"Lines": [dict({"Highlighted": ""}, **ln) for ln in s["Code"]["Lines"]]}
            finds.append(f)
        cases.append({"name": "integration " + res["Target"],
                      "config": "trivy-secret.yaml", "input": res["Target"], "path": res["Target"],
                      "want": {"FilePath": res["Target"], "Findings": finds},
                      "ref": "integration/testdata/secrets.json.golden"})
    copy_data(["deploy.sh", "trivy-secret.yaml"], os.path.join(base, "fixtures/repo/secrets"),
              os.path.join(HERE, "integration"))
    # the golden report itself (the bytes `trivy -f json` wrote with -update,
    # integration/integration_test.go:244-247), for the report writer's test
    copy_data(["secrets.json.golden"], base, os.path.join(HERE, "integration"))
    return cases


def main():
    env = gen_builtin_rules.parse_consts(open(os.path.join(REF, "pkg/fanal/secret/builtin-rules.go")).read())
    sc = scanner_cases(env)
    an, req = analyzer_cases(env)
    it = integration_cases()
    for name, data in (("scanner_cases.json", sc), ("analyzer_cases.json", {"analyze": an, "required": req}),
                       ("integration_cases.json", it)):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f, indent=1, ensure_ascii=False)
            f.write("\n")
    print("scanner cases:", len(sc), "analyzer:", len(an), "required:", len(req), "integration:", len(it))


if __name__ == "__main__":
    main()
