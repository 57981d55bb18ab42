"""Hydra-style config composition for `train.py experiment=...` without Hydra/OmegaConf.

Implements the subset of Hydra 1.3 / OmegaConf 2.3 semantics the reference's hot-path configs
rely on (configs/config.yaml, configs/experiment/dnabert2/*.yaml, configs/pipeline/bert_hg38.yaml
and the group files they pull in):
  * defaults lists with `_self_`, `group: option`, absolute `/group: option`, option lists
    (`/callbacks: [base, checkpoint]`), `override /group: option`, `group: null`, optional entries;
  * `# @package _global_` / `# @package a.b` headers (default package = the group path);
  * command-line overrides: group choices `experiment=dnabert2/x`, values `a.b=v`, `+a.b=v`,
    `++a.b=v`, deletions `~a.b`;
  * lazy interpolation: `${a.b}`, relative `${.x}` / `${..x}`, resolvers `eval` (Python eval,
    as registered at train.py:47), `div_up` (:48) and `now`; `???` is a missing value that only
    fails when read. Values are resolved on access, so `train.gpu_mem` (which shells out to
    nvidia-smi, dnabert2_hg38_pretrain.yaml:89) never runs unless something reads it.
"""
import copy
import datetime
import math
import os
import re

import yaml

MISSING = "???"


class ConfigError(RuntimeError):
    pass


# ------------------------------------------------------------------------------------- loading
class _Loader(yaml.SafeLoader):
    """SafeLoader + OmegaConf's float rule: `5e-4` / `1E6` (no dot) are floats, not strings."""


_Loader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    re.compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
                  |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
                  |\.[0-9_]+(?:[eE][-+][0-9]+)?
                  |[-+]?\.(?:inf|Inf|INF)
                  |\.(?:nan|NaN|NAN))$""", re.X),
    list("-+0123456789."))


def _yaml(text):
    return yaml.load(text, Loader=_Loader)


def _read(path):
    text = open(path).read()
    pkg = None
    for line in text.splitlines():
        s = line.strip()
        if s.startswith("#") and "@package" in s:
            pkg = s.split("@package", 1)[1].strip()
            break
        if s and not s.startswith("#"):
            break
    data = _yaml(text) or {}
    if not isinstance(data, dict):
        raise ConfigError(f"{path}: top level must be a mapping")
    return data, pkg


def _set(d, dotted, value, create=True):
    keys = dotted.split(".") if dotted else []
    cur = d
    for k in keys[:-1]:
        if k not in cur or not isinstance(cur[k], dict):
            if not create and k not in cur:
                raise ConfigError(f"override of missing key '{dotted}' (use +{dotted}=...)")
            cur[k] = {}
        cur = cur[k]
    if not keys:
        raise ConfigError("empty key")
    if not create and keys[-1] not in cur:
        raise ConfigError(f"override of missing key '{dotted}' (use +{dotted}=...)")
    cur[keys[-1]] = value


def _merge(dst, src):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _wrap(pkg, data):
    if not pkg:
        return copy.deepcopy(data)
    out = {}
    _set(out, pkg, copy.deepcopy(data))
    return out


class _Defaults:
    """Two passes over the defaults tree: collect group choices (+ `override`), then expand."""

    def __init__(self, root):
        self.root = root

    def _path(self, group, option):
        p = os.path.join(self.root, group, f"{option}.yaml") if group else \
            os.path.join(self.root, f"{option}.yaml")
        if not os.path.exists(p):
            raise ConfigError(f"config not found: {p}")
        return p

    @staticmethod
    def _entries(data, cur_group):
        """Normalised (kind, group, options, optional) from a file's defaults list."""
        out = []
        for e in data.get("defaults", []) or []:
            if isinstance(e, str):
                out.append(("self", None, None, False) if e == "_self_" else
                           ("file", cur_group, [e], False))
                continue
            if not isinstance(e, dict) or len(e) != 1:
                raise ConfigError(f"bad defaults entry {e!r}")
            (k, v), = e.items()
            k = k.strip()
            kind, optional = "group", False
            if k.startswith("override "):
                kind, k = "override", k[len("override "):].strip()
            if k.startswith("optional "):
                optional, k = True, k[len("optional "):].strip()
            group = k[1:] if k.startswith("/") else (f"{cur_group}/{k}" if cur_group else k)
            opts = None if v is None else (list(v) if isinstance(v, list) else [str(v)])
            out.append((kind, group, opts, optional))
        return out

    def collect(self, path, cur_group, choices, overrides, cli, seen):
        """choices: first default seen per group; overrides: `override` entries + CLI choices
        (CLI always wins)."""
        data, _ = _read(path)
        for kind, group, opts, optional in self._entries(data, cur_group):
            if kind == "self":
                continue
            if kind == "override":
                if group not in cli:
                    overrides[group] = opts
                continue
            if kind == "file":
                self.collect(self._path(group, opts[0]), group, choices, overrides, cli, seen)
                continue
            choices.setdefault(group, opts)
            sel = overrides.get(group, choices[group])
            for o in sel or []:
                key = (group, o)
                if key in seen:
                    continue
                seen.add(key)
                p = os.path.join(self.root, group, f"{o}.yaml")
                if os.path.exists(p):
                    self.collect(p, group, choices, overrides, cli, seen)
                elif not optional:
                    raise ConfigError(f"config not found: {p}")

    def expand(self, path, cur_group, final, out, default_pkg):
        data, pkg = _read(path)
        pkg = default_pkg if pkg is None else ("" if pkg == "_global_" else pkg)
        body = {k: v for k, v in data.items() if k != "defaults"}
        entries = self._entries(data, cur_group)
        if not any(e[0] == "self" for e in entries):
            entries.append(("self", None, None, False))
        for kind, group, opts, optional in entries:
            if kind == "self":
                out.append(_wrap(pkg, body))
            elif kind == "override":
                continue
            elif kind == "file":
                self.expand(self._path(group, opts[0]), group, final, out, pkg)
            else:
                for o in final.get(group) or []:
                    p = os.path.join(self.root, group, f"{o}.yaml")
                    if not os.path.exists(p):
                        if optional:
                            continue
                        raise ConfigError(f"config not found: {p}")
                    self.expand(p, group, final, out, group.replace("/", "."))


def compose(config_dir, config_name="config", overrides=()):
    """-> Config (lazy-resolving view) of config_dir/config_name.yaml with CLI overrides."""
    config_dir = os.path.abspath(config_dir)
    group_ov, value_ov = {}, []
    for ov in overrides:
        key = ov.split("=", 1)[0]
        bare = key.lstrip("+~")
        if "=" in ov and not key.startswith(("+", "~")) and \
                os.path.isdir(os.path.join(config_dir, bare.replace(".", "/"))):
            val = ov.split("=", 1)[1]
            group_ov[bare] = None if val in ("null", "") else [v.strip() for v in
                                                              val.strip("[]").split(",")]
        else:
            value_ov.append(ov)
    d = _Defaults(config_dir)
    primary = os.path.join(config_dir, f"{config_name}.yaml")
    choices, ov = {}, dict(group_ov)
    for _ in range(4):  # a chosen option may carry further `override`s: iterate to a fixpoint
        choices, ov2 = {}, dict(ov)
        d.collect(primary, "", choices, ov2, group_ov, set())
        if ov2 == ov:
            break
        ov = ov2
    final = dict(choices)
    final.update(ov)
    parts = []
    d.expand(primary, "", final, parts, "")
    cfg = {}
    for p in parts:
        _merge(cfg, p)
    for ov in value_ov:
        if ov.startswith("~"):
            keys = ov[1:].split("=", 1)[0].split(".")
            cur = cfg
            for k in keys[:-1]:
                cur = cur.get(k, {})
            cur.pop(keys[-1], None)
            continue
        key, val = ov.split("=", 1)
        force = key.startswith("++")
        add = key.startswith("+") and not force
        key = key.lstrip("+")
        v = _yaml(val) if val != "" else None
        _set(cfg, key, v, create=add or force or _has(cfg, key) or _parent_exists(cfg, key))
    cfg.setdefault("hydra_choices", {k: v for k, v in final.items()})
    return Config(cfg)


def _has(d, dotted):
    cur = d
    for k in dotted.split("."):
        if not isinstance(cur, dict) or k not in cur:
            return False
        cur = cur[k]
    return True


def _parent_exists(d, dotted):
    keys = dotted.split(".")
    return len(keys) == 1 or _has(d, ".".join(keys[:-1]))


# ------------------------------------------------------------------------------ interpolation
_INTERP = re.compile(r"\$\{")


def _find_close(s, i):
    depth = 0
    j = i
    while j < len(s):
        if s.startswith("${", j):
            depth += 1
            j += 2
            continue
        if s[j] == "}":
            depth -= 1
            if depth == 0:
                return j
        j += 1
    raise ConfigError(f"unbalanced interpolation in {s!r}")


class Config:
    """Read-only view over a composed dict; attribute/item access resolves interpolations."""

    RESOLVERS = {
        "eval": lambda s: eval(s),  # noqa: S307 -- same semantics as the reference's resolver
        "div_up": lambda x, y: (int(x) + int(y) - 1) // int(y),
        "now": lambda fmt: datetime.datetime.now().strftime(fmt),
    }

    def __init__(self, data, root=None, path=()):
        object.__setattr__(self, "_d", data)
        object.__setattr__(self, "_root", root if root is not None else data)
        object.__setattr__(self, "_path", path)

    # -- mapping interface
    def keys(self):
        return self._d.keys()

    def items(self):
        return [(k, self[k]) for k in self._d]

    def __iter__(self):
        return iter(self._d)

    def __len__(self):
        return len(self._d)

    def __contains__(self, k):
        return k in self._d

    def get(self, k, default=None):
        return self[k] if k in self._d else default

    def __getitem__(self, k):
        if k not in self._d:
            raise KeyError(".".join(self._path + (str(k),)))
        return self._resolve(self._d[k], self._path + (k,))

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)

    def __setattr__(self, k, v):
        self._d[k] = v

    def __setitem__(self, k, v):
        self._d[k] = v

    def pop(self, k, default=None):
        return self._d.pop(k, default)

    def to_container(self, resolve=True, skip_errors=False):
        def conv(v, path):
            if isinstance(v, dict):
                return {k: conv(v[k], path + (k,)) for k in v}
            if isinstance(v, list):
                return [conv(x, path + (i,)) for i, x in enumerate(v)]
            if resolve:
                try:
                    r = self._resolve(v, path)
                except Exception as e:  # noqa: BLE001
                    if not skip_errors:
                        raise
                    return f"<unresolved: {e}>"
                return r.to_container(resolve, skip_errors) if isinstance(r, Config) else r
            return v
        return conv(self._d, self._path)

    # -- resolution
    def _lookup(self, dotted, here):
        if dotted.startswith("."):
            n = len(dotted) - len(dotted.lstrip("."))
            base = list(here[:-1])[: max(0, len(here) - n)] if n else list(here)
            rest = dotted[n:]
            keys = base + (rest.split(".") if rest else [])
        else:
            keys = dotted.split(".")
        cur = self._root
        for k in keys:
            if isinstance(cur, list):
                cur = cur[int(k)]
            elif isinstance(cur, dict) and k in cur:
                cur = cur[k]
            else:
                raise ConfigError(f"interpolation key '{dotted}' not found")
        return self._resolve(cur, tuple(keys))

    def _resolve(self, v, path):
        if isinstance(v, dict):
            return Config(v, self._root, path)
        if isinstance(v, list):
            return [self._resolve(x, path + (i,)) for i, x in enumerate(v)]
        if isinstance(v, str):
            if v == MISSING:
                raise ConfigError(f"missing mandatory value: {'.'.join(map(str, path))}")
            if "${" in v:
                return self._interp(v, path)
        return v

    def _interp(self, s, path):
        m = _INTERP.search(s)
        if m and m.start() == 0 and _find_close(s, 0) == len(s) - 1:
            return self._one(s[2:-1], path)
        out, i = "", 0
        while True:
            m = _INTERP.search(s, i)
            if not m:
                return out + s[i:]
            j = _find_close(s, m.start())
            out += s[i:m.start()] + str(self._one(s[m.start() + 2:j], path))
            i = j + 1

    def _one(self, expr, path):
        expr = expr.strip()
        head = re.match(r"^([A-Za-z_][A-Za-z0-9_]*):", expr)
        if head and head.group(1) in self.RESOLVERS:
            name, argstr = head.group(1), expr[head.end():]
            args = self._split_args(argstr)
            vals = []
            for a in args:
                a = a.strip()
                r = self._interp(a, path) if "${" in a else a
                if isinstance(r, str):
                    if len(r) >= 2 and r[0] == r[-1] and r[0] in "'\"":
                        r = r[1:-1]
                    elif name != "eval":
                        r = _yaml(r)
                vals.append(r)
            if name == "eval":
                return self.RESOLVERS["eval"](",".join(str(x) for x in vals))
            return self.RESOLVERS[name](*vals)
        return self._lookup(expr, path)

    @staticmethod
    def _split_args(s):
        out, depth, cur, quote = [], 0, "", None
        for ch in s:
            if quote:
                cur += ch
                if ch == quote:
                    quote = None
                continue
            if ch in "'\"":
                quote = ch
            elif ch in "([{":
                depth += 1
            elif ch in ")]}":
                depth -= 1
            elif ch == "," and depth == 0:
                out.append(cur)
                cur = ""
                continue
            cur += ch
        out.append(cur)
        return out

    def __repr__(self):
        return f"Config({self.to_container(resolve=False)!r})"


def math_ok():  # keep `math` importable inside eval'd expressions, like Python's builtins
    return math
