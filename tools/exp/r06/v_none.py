# no edit: the working tree as is (EXTRA flags select the variant)
