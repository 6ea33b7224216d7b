from .backbone import BACKBONES, BackboneFactory
from .generic import BaseModel, Classifier, CoordinateRegressor


def list_backbones(family: str | None = None) -> list[str]:
    return BackboneFactory.list_backbones(family)


__all__ = ["BACKBONES", "BackboneFactory", "BaseModel", "Classifier", "CoordinateRegressor", "list_backbones"]
