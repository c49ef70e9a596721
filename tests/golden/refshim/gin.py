"""Minimal stand-in for gin-config (absent here) used only to path-import the
reference modules in make_golden.py.  Bindings from the .gin files are applied
by hand there; this stub only provides identity decorators."""


def configurable(*args, **kwargs):
    if len(args) == 1 and callable(args[0]) and not kwargs:
        return args[0]
    return lambda f: f


def external_configurable(*args, **kwargs):
    return configurable(*args, **kwargs)


def constant(*args, **kwargs):
    return None


def enter_interactive_mode():
    return None


def parse_config_files_and_bindings(*args, **kwargs):
    raise RuntimeError("gin stub: bindings are applied explicitly")


def REQUIRED():  # noqa: N802
    return None
