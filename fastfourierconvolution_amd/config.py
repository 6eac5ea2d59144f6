"""Minimal stand-in for the reference's ``Config`` singleton (config/params.py:8-28): only the
``DEBUG`` flag read by ``Print`` / ``debug_print`` (layers/print_layer.py:10-12) is on the path."""


class Config:
    _instance = None
    DEBUG = False

    @classmethod
    def shared(cls):
        if cls._instance is None:
            cls._instance = cls()
        return cls._instance
