"""Test-only stub: the reference imports gymnasium only for a type annotation."""


class Env:
    pass
