OBJECT = "py/object"
