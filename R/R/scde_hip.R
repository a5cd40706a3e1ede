# scde_hip.R -- R wrappers for the fused device path of libscde_hip (R/src/scde_hip_shim.c).
#
# With the shim installed, the reference's own scde.posteriors / scde.expression.difference
# (R/functions.R:566, 304) already run on the GPU through the layer-1 .Call symbols.  These
# functions keep exactly those signatures but hand the whole call to the device in one .Call:
# unique-count tables, both groups' posteriors, the ratio posterior, the summary and BH run
# in HBM (scde_expression_difference_host; the batch-corrected branch, R/functions.R:321-399, through
# scde_expression_difference_batch_host).  Arguments the fused path does not cover (batch.models of
# another model type than models, scde.posteriors with a batch) go to the reference implementation,
# saved as .scde.ref.* first, which runs over the layer-1 .Call symbols of the same library.

.scde.model.matrix <- function(models) {
    # R/functions.R:601-604 (mm), with the flags R/functions.R:595-598 derives
    mm <- matrix(NA, nrow(models), 12)
    cols <- c("conc.b", "conc.a", "fail.r", "corr.b", "corr.a", "corr.theta", "corr.ltheta.b", "corr.ltheta.t",
              "corr.ltheta.m", "corr.ltheta.s", "corr.ltheta.r", "conc.a2")
    for (j in seq_along(cols)) if (cols[j] %in% colnames(models)) mm[, j] <- models[, cols[j]]
    list(mm = mm, localtheta = "corr.ltheta.b" %in% colnames(models), squarelogit = "conc.a2" %in% colnames(models))
}

if (!exists(".scde.ref.expression.difference")) .scde.ref.expression.difference <- scde.expression.difference
if (!exists(".scde.ref.posteriors")) .scde.ref.posteriors <- scde.posteriors

scde.expression.difference <- function(models, counts, prior, groups = NULL, batch = NULL, n.randomizations = 150,
                                       n.cores = 10, batch.models = models, return.posteriors = FALSE,
                                       expectation = 0, verbose = 0) {
    if (!all(rownames(models) %in% colnames(counts))) {
        stop("ERROR: provided count data does not cover all of the cells specified in the model matrix")
    }
    counts <- as.matrix(counts[, match(rownames(models), colnames(counts))])
    if (is.null(groups)) {
        groups <- as.factor(attr(models, "groups"))
        if (is.null(groups)) stop("ERROR: groups factor is not provided, and models structure is lacking groups attribute")
        names(groups) <- rownames(models)
    }
    if (length(levels(groups)) != 2) {
        stop(paste("ERROR: wrong number of levels in the grouping factor (", paste(levels(groups), collapse = " "),
                   "), but must be two.", sep = ""))
    }
    # the reference splits the model rows by position, tapply(seq_len(nrow(models)), groups, ...)
    # (R/functions.R:355, 372): the codes go by position too, never by name
    if (length(groups) != nrow(models)) stop("arguments must have same length")
    gcodes <- as.integer(groups)
    correct.batch <- !is.null(batch) && length(levels(batch)) > 1  # R/functions.R:321-330
    storage.mode(counts) <- "integer"
    m <- .scde.model.matrix(models)
    m$mm[, 5] <- pmax(m$mm[, 5], 1e-10)  # R/functions.R:579-583
    marginals <- log(pmax(10^prior$x - 1, 0))
    rv <- seq(prior$x[1] - prior$x[length(prior$x)], prior$x[length(prior$x)] - prior$x[1],
              length = length(prior$x) * 2 - 1)
    name.jp <- function(j) {
        rownames(j) <- rownames(counts)
        colnames(j) <- as.character(exp(marginals))
        j
    }
    name.tab <- function(t) {
        res <- as.data.frame(t)
        colnames(res) <- c("lb", "mle", "ub", "ce", "Z", "cZ")
        rownames(res) <- rownames(counts)
        res
    }
    if (correct.batch) {
        batch <- as.factor(batch)
        if (length(batch) != nrow(models)) stop("arguments must have same length")
        bm <- .scde.model.matrix(batch.models)
        if (bm$localtheta != m$localtheta || bm$squarelogit != m$squarelogit || nrow(bm$mm) != nrow(m$mm) ||
            !identical(rownames(batch.models), rownames(models))) {
            # batch.models of another model type, or of other cells / another row order: the
            # reference's batch posteriors reorder the counts by rownames(batch.models) and pair
            # batch[i] with batch.models row i (R/functions.R:356, 570, 573-574), which the fused
            # call (one count matrix in models' order) does not express -- the reference glue over
            # the layer-1 symbols
            return(.scde.ref.expression.difference(models, counts, prior, groups, batch, n.randomizations, n.cores,
                                                   batch.models, return.posteriors, expectation, verbose))
        }
        bgti <- table(groups, batch)  # R/functions.R:336-349
        bgti.ft <- fisher.test(bgti)
        if (verbose) {
            cat("controlling for batch effects. interaction:\n")
            print(bgti)
        }
        if (bgti.ft$p.value < 1e-3) {
            cat("WARNING: strong interaction between groups and batches! Correction may be ineffective:\n")
            print(bgti.ft)
        }
        bm$mm[, 5] <- pmax(bm$mm[, 5], 1e-10)
        x <- .Call("scde_hip_expression_difference_batch", m$mm, bm$mm, counts, prior$x, prior$y, gcodes,
                   as.integer(batch), length(levels(batch)), n.randomizations, n.cores, m$localtheta, m$squarelogit,
                   expectation, return.posteriors, PACKAGE = "scde")
        out <- list(batch.adjusted = name.tab(x$batch.adjusted), results = name.tab(x$results),
                    batch.effect = name.tab(x$batch.effect))
        if (!return.posteriors) return(out)
        ratio <- x$ratio
        dimnames(ratio) <- list(rownames(counts), as.character(rv))
        rv2 <- as.numeric(colnames(ratio))  # the second level's prior x (R/functions.R:391)
        rv2 <- seq(rv2[1] - rv2[length(rv2)], rv2[length(rv2)] - rv2[1], length = length(rv2) * 2 - 1)
        aratio <- x$adj.ratio
        dimnames(aratio) <- list(rownames(counts), as.character(rv2))
        jp <- lapply(list(x$jp1, x$jp2), name.jp)
        names(jp) <- levels(groups)
        return(c(out, list(difference.posterior = ratio, batch.adjusted.difference.posterior = aratio,
                           joint.posteriors = jp)))
    }
    x <- .Call("scde_hip_expression_difference", m$mm, counts, prior$x, prior$y, gcodes, n.randomizations, n.cores,
               m$localtheta, m$squarelogit, expectation, return.posteriors, PACKAGE = "scde")
    res <- name.tab(x$results)
    if (!return.posteriors) return(res)
    jp <- lapply(list(x$jp1, x$jp2), name.jp)
    names(jp) <- levels(groups)
    ratio <- x$ratio
    rownames(ratio) <- rownames(counts)
    colnames(ratio) <- as.character(rv)
    list(results = res, difference.posterior = ratio, joint.posteriors = jp)
}

scde.posteriors <- function(models, counts, prior, n.randomizations = 100, batch = NULL, composition = NULL,
                            return.individual.posteriors = FALSE, return.individual.posterior.modes = FALSE,
                            ensemble.posterior = FALSE, n.cores = 20) {
    if (!all(rownames(models) %in% colnames(counts))) {
        stop("ERROR: provided count data does not cover all of the cells specified in the model matrix")
    }
    batchil <- NULL
    if (!is.null(batch)) {  # R/functions.R:568-571: batch-sampled posteriors
        if (is.null(composition)) stop("ERROR: group composition must be provided if the batch argument is passed")
        batchil <- tapply(c(1:nrow(models)) - 1, batch, I)
        composition <- as.integer(composition)
    }
    counts <- as.matrix(counts[, match(rownames(models), colnames(counts)), drop = FALSE])
    storage.mode(counts) <- "integer"
    marginals <- log(pmax(10^prior$x - 1, 0))
    postflag <- 0
    if (return.individual.posteriors) {
        postflag <- if (return.individual.posterior.modes) 3 else 2
    } else if (return.individual.posterior.modes) {
        postflag <- 1
    }
    m <- .scde.model.matrix(models)
    m$mm[, 5] <- pmax(m$mm[, 5], 1e-10)
    if (any(models$corr.a < 1e-10)) {  # R/functions.R:579-583
        cat("WARNING: the following cells have negatively-correlated or 0-slope fits: ",
            paste(rownames(models)[models$corr.a < 1e-10], collapse = " "), ". Setting slopes to 1e-10.\n")
    }
    x <- .Call("scde_hip_posteriors", m$mm, counts, prior$x, n.randomizations, n.cores, m$localtheta, m$squarelogit,
               postflag, ensemble.posterior, batchil, composition, PACKAGE = "scde")
    if (!is.null(batch) && postflag == 3) postflag <- 0  # the reference's batch call returns jp only
    name.jp <- function(j) {
        rownames(j) <- rownames(counts)
        colnames(j) <- as.character(exp(marginals))
        j
    }
    if (postflag == 0) return(name.jp(x))
    x$jp <- name.jp(x$jp)
    if (!is.null(x$modes)) {
        rownames(x$modes) <- rownames(counts)
        colnames(x$modes) <- rownames(models)
    }
    if (!is.null(x$post)) {
        names(x$post) <- rownames(models)
        x$post <- lapply(x$post, name.jp)
    }
    x
}

# pagoda.varnorm's mode and weight computation (R/functions.R:1414-1507) in one call; returns
# list(avmodes, modes (one column per batch level, or NULL), matw, bmatw)
scde.hip.varnorm.weights <- function(models, counts, prior, batch = NULL, n.randomizations = 100, n.cores = 1,
                                     use.expected.value = TRUE) {
    counts <- as.matrix(counts[, match(rownames(models), colnames(counts)), drop = FALSE])
    storage.mode(counts) <- "integer"
    m <- .scde.model.matrix(models)
    nb <- 0
    codes <- integer(0)
    if (!is.null(batch)) {
        batch <- as.factor(batch)
        bt <- table(batch)
        if (any(bt < 2)) batch[batch %in% names(bt)[bt < 2]] <- names(bt)[which.max(bt)]  # R/functions.R:1404-1410
        batch <- droplevels(batch)
        nb <- length(levels(batch))
        codes <- as.integer(batch)
    }
    x <- .Call("scde_hip_varnorm_weights", m$mm, counts, prior$x, n.randomizations, n.cores, m$localtheta,
               m$squarelogit, codes, nb, use.expected.value, PACKAGE = "scde")
    avmodes <- x$modes[, 1]
    names(avmodes) <- rownames(counts)
    modes <- if (nb > 1) x$modes[, -1, drop = FALSE] else NULL
    if (!is.null(modes)) dimnames(modes) <- list(rownames(counts), levels(batch))
    dimnames(x$matw) <- list(rownames(counts), rownames(models))
    if (!is.null(x$bmatw)) dimnames(x$bmatw) <- list(rownames(counts), rownames(models))
    list(avmodes = avmodes, modes = modes, matw = x$matw, bmatw = x$bmatw)
}
