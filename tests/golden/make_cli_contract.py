"""Record the CLI contract of the reference's do-compress.sh as DATA in
manifest.json (run in the build container, where /root/reference exists):
the script's sha256, the usage check (no argument -> message, exit 1) and
the argv of every `./main` call it makes, with the file names expressed
through the script's own variables ({f} = "$1").  tests/test_gpu_cli.py
replays that argv sequence against this build's `main`; tests/test_oracle.py
re-derives the contract from the reference script when it is present.

  python tests/golden/make_cli_contract.py
"""
import hashlib
import json
import os
import re
import shlex

HERE = os.path.dirname(os.path.abspath(__file__))
SCRIPT = "/root/reference/do-compress.sh"


def derive(text):
    """The contract of a do-compress.sh text: variables assigned from $1 and
    from each other (`x="${fname}.vcfc"`), the `./main` calls with their
    arguments resolved to templates over {f}, and the usage message."""
    env = {"1": "{f}"}
    calls, usage = [], None
    for raw in text.splitlines():
        line = raw.strip()
        m = re.match(r'^([A-Za-z_][A-Za-z0-9_]*)="?(.*?)"?$', line)
        if m and "=" in line and not line.startswith(("if", "./", "echo")):
            env[m.group(1)] = re.sub(r'\$\{?([A-Za-z0-9_]+)\}?', lambda v: env[v.group(1)], m.group(2))
            continue
        m = re.match(r'^echo "(.*)"$', line)
        if m and usage is None:
            usage = m.group(1) + "\n"
            continue
        if line.startswith("./main "):
            cmd = line.split("|")[0].replace("2>&1", "")
            argv = [re.sub(r'\$\{?([A-Za-z0-9_]+)\}?', lambda v: env[v.group(1)], a) for a in shlex.split(cmd)[1:]]
            log = None
            tee = re.search(r'tee\s+(\S+)', line)
            if tee:
                log = tee.group(1)
            calls.append({"argv": argv, "log": log})
    return {"usage_stdout": usage, "usage_rc": 1, "calls": calls}


def main():
    with open(SCRIPT, "rb") as f:
        data = f.read()
    c = derive(data.decode())
    c["script_sha256"] = hashlib.sha256(data).hexdigest()
    p = os.path.join(HERE, "manifest.json")
    with open(p) as f:
        man = json.load(f)
    man["do_compress"] = c
    with open(p, "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print(json.dumps(c, indent=1))


if __name__ == "__main__":
    main()
